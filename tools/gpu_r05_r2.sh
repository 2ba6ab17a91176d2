#!/bin/bash
# Round-5 GPU step R (r2): mat_mult_q7 with two staging register sets (MI355X_Q7_RING=2, loads two K
# steps ahead), alone and with 256 x 128 tiles, against the default: the q7 GEMM GPU tests on each
# variant, then three alternating bench lines.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2; mkdir -p $O
step() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step rc=$rc: $*"; exit $rc; }; }
show() { python -c "import json;d=json.load(open('$1'));p=d['parity'];print('$2',d['value'],d['roofline']['frac'],d['roofline']['avg_kernel_ms'],p.get('bit_exact',p) if isinstance(p,dict) else p)"; }
lib() { [ $1 = default ] && echo cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so || echo cmsis-dsp_amd/lib/variants/lib_$1.so; }
PT="-x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
for v in q7ring2 q7ring2bn128; do
  CMSISDSP_MI355X_LIB=$(lib $v) step 300 python -u -m pytest tests/test_gpu_rfft_fir_mat.py -m gpu -k q7 $PT > $O/t_$v.log 2>&1
  echo "$v tests: $(tail -1 $O/t_$v.log)"
done
for rep in 1 2 3; do
for v in default q7ring2 q7ring2bn128; do
  CMSISDSP_MI355X_LIB=$(lib $v) step 200 python -u bench.py --workload mat_mult_q7 --no-cpu-baseline > $O/q7_${v}_$rep.json 2> $O/q7_${v}_$rep.err
  show $O/q7_${v}_$rep.json q7_$v
done
done
echo all-ok
