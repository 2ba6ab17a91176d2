#!/bin/bash
# Round-5 GPU step F: software-pipelined q7 / q15 LDS-DMA GEMMs (fragments of step kt+1 read under step
# kt's MFMAs): bit-exact tests, then A/B against the default kernel, same box.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/f1; mkdir -p $O
step() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step rc=$rc: $*"; exit $rc; }; }
show() { python -c "import json;d=json.load(open('$1'));p=d['parity'];print('$2',d['value'],d['roofline']['frac'],d['roofline']['avg_kernel_ms'],p.get('bit_exact',p) if isinstance(p,dict) else p)"; }
lib() { [ $1 = default ] && echo cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so || echo cmsis-dsp_amd/lib/variants/lib_$1.so; }
PT="-x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
for v in q7p1 q7p2; do
  CMSISDSP_MI355X_LIB=$(lib $v) step 300 python -u -m pytest tests/test_gpu_rfft_fir_mat.py tests/test_gpu_runtime.py -k q7 $PT > $O/t_$v.log 2>&1
  echo "$v: $(tail -1 $O/t_$v.log)"
done
CMSISDSP_MI355X_LIB=$(lib q15p1) step 300 python -u -m pytest tests/test_gpu_rfft_fir_mat.py -k "mat_mult_fixed or mat_mult_fast" $PT > $O/t_q15p1.log 2>&1
echo "q15p1: $(tail -1 $O/t_q15p1.log)"
CMSISDSP_MI355X_LIB=$(lib q15p2) step 300 python -u -m pytest tests/test_gpu_rfft_fir_mat.py -k "mat_mult_fixed or mat_mult_fast" $PT > $O/t_q15p2.log 2>&1
echo "q15p2: $(tail -1 $O/t_q15p2.log)"
for rep in 1 2; do
for v in default q7p1 q7p2; do
  CMSISDSP_MI355X_LIB=$(lib $v) step 200 python -u bench.py --workload mat_mult_q7 --no-cpu-baseline > $O/q7_$v.json 2> $O/q7_$v.err
  show $O/q7_$v.json q7_$v
done
for v in default q15p1 q15p2; do
  CMSISDSP_MI355X_LIB=$(lib $v) step 200 python -u bench.py --workload mat_mult_q15 --no-cpu-baseline > $O/q15_$v.json 2> $O/q15_$v.err
  show $O/q15_$v.json q15_$v
done
done
echo all-ok
