#!/bin/bash
# Round-5 GPU step J: q31 GEMM row sums by v_dot4 over the cut planes; q7 GEMM with transposed accumulators (operands swapped in the MFMA, the
# epilogue packs 4 outputs per LDS dword): bit-exact tests, then A/B against the default.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/j1; mkdir -p $O
step() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step rc=$rc: $*"; exit $rc; }; }
show() { python -c "import json;d=json.load(open('$1'));p=d['parity'];print('$2',d['value'],d['roofline']['frac'],d['roofline']['avg_kernel_ms'],p.get('bit_exact',p) if isinstance(p,dict) else p)"; }
lib() { [ $1 = default ] && echo cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so || echo cmsis-dsp_amd/lib/variants/lib_$1.so; }
PT="-x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
CMSISDSP_MI355X_LIB=$(lib q7tepi) step 300 python -u -m pytest tests/test_gpu_rfft_fir_mat.py tests/test_gpu_runtime.py -k q7 $PT > $O/t_q7tepi.log 2>&1
echo "q7tepi tests: $(tail -1 $O/t_q7tepi.log)"
CMSISDSP_MI355X_LIB=$(lib q31rsdot) step 300 python -u -m pytest tests/test_gpu_rfft_fir_mat.py -k "mat_mult_fixed or mat_mult_fast" $PT > $O/t_q31rsdot.log 2>&1
echo "q31rsdot tests: $(tail -1 $O/t_q31rsdot.log)"
for rep in 1 2 3; do
for v in default q31rsdot; do
  CMSISDSP_MI355X_LIB=$(lib $v) step 200 python -u bench.py --workload mat_mult_q31 --no-cpu-baseline > $O/q31_$v.json 2> $O/q31_$v.err
  show $O/q31_$v.json q31_$v
done
for v in default q7tepi; do
  CMSISDSP_MI355X_LIB=$(lib $v) step 200 python -u bench.py --workload mat_mult_q7 --no-cpu-baseline > $O/q7_$v.json 2> $O/q7_$v.err
  show $O/q7_$v.json q7_$v
done
done
echo all-ok
