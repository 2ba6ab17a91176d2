#!/bin/bash
# Round-5 GPU step L: f32 GEMM with an unpadded, XOR-swizzled A tile (32 KiB of LDS: five
# workgroups per CU) — fmaf-chain bit-exact tests, then A/B against the default, same box.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/l1; mkdir -p $O
step() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step rc=$rc: $*"; exit $rc; }; }
lib() { [ $1 = default ] && echo cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so || echo cmsis-dsp_amd/lib/variants/lib_$1.so; }
PT="-x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
CMSISDSP_MI355X_LIB=$(lib f32w5) step 300 python -u -m pytest tests/test_gpu_rfft_fir_mat.py -k "mat_mult_f32 or mat_f32" $PT > $O/t_f32w5.log 2>&1
echo "f32w5 tests: $(tail -1 $O/t_f32w5.log)"
for rep in 1 2 3; do
for v in default f32w5; do
  CMSISDSP_MI355X_LIB=$(lib $v) step 200 python -u bench.py --workload mat_mult_f32 --no-cpu-baseline > $O/f32_$v.json 2> $O/f32_$v.err
  python -c "import json;d=json.load(open('$O/f32_$v.json'));print('f32_$v',d['value'],d['roofline']['frac'],d['roofline']['avg_kernel_ms'],d['parity']['fmaf_chain_bit_exact'])"
done
done
echo all-ok
