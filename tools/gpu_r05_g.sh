#!/bin/bash
# Round-5 GPU step G: f32 GEMM tile order / start stagger A/B (configs[4]), same box.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/g1; mkdir -p $O
step() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step rc=$rc: $*"; exit $rc; }; }
lib() { [ $1 = default ] && echo cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so || echo cmsis-dsp_amd/lib/variants/lib_$1.so; }
for rep in 1 2 3; do
for v in default f32x0 f32st16 f32st32; do
  CMSISDSP_MI355X_LIB=$(lib $v) step 200 python -u bench.py --workload mat_mult_f32 --no-cpu-baseline > $O/f32_$v.json 2> $O/f32_$v.err
  python -c "import json;d=json.load(open('$O/f32_$v.json'));print('f32_$v',d['value'],d['roofline']['frac'],d['roofline']['avg_kernel_ms'],d['parity']['fmaf_chain_bit_exact'])"
done
done
echo all-ok
