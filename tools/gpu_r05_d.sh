#!/bin/bash
# Round-5 GPU step D: step C (q7 / q15 LDS-DMA variants, RFFT p-scratch mapping) plus the f32 GEMM
# tile-order / K-tile variants (mat_mult_f32 configs[4]), same box.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/d1; mkdir -p $O
step() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step rc=$rc: $*"; exit $rc; }; }
show() { python -c "import json;d=json.load(open('$1'));print('$2',d['value'],d['roofline']['frac'],d['roofline']['avg_kernel_ms'],d['parity'].get('bit_exact', d['parity']))"; }
lib() { [ $1 = default ] && echo cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so || echo cmsis-dsp_amd/lib/variants/lib_$1.so; }
CMSISDSP_MI355X_LIB=$(lib q15dma) step 300 python -u -m pytest tests/test_gpu_rfft_fir_mat.py \
  -k "mat_mult_fixed or mat_mult_fast" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/q15dma_tests.log 2>&1
tail -2 $O/q15dma_tests.log
for rep in 1 2; do
for v in default q7dma q7dmanoepi q7kt128 q7noepi; do
  CMSISDSP_MI355X_LIB=$(lib $v) step 200 python -u bench.py --workload mat_mult_q7 --no-cpu-baseline > $O/q7_$v.json 2> $O/q7_$v.err
  show $O/q7_$v.json q7_$v
done
for v in default q15dma; do
  CMSISDSP_MI355X_LIB=$(lib $v) step 200 python -u bench.py --workload mat_mult_q15 --no-cpu-baseline > $O/q15_$v.json 2> $O/q15_$v.err
  show $O/q15_$v.json q15_$v
done
for v in default f32x1 f32bk32 f32x1bk32; do
  CMSISDSP_MI355X_LIB=$(lib $v) step 200 python -u bench.py --workload mat_mult_f32 --no-cpu-baseline > $O/f32_$v.json 2> $O/f32_$v.err
  show $O/f32_$v.json f32_$v
done
for v in default rfTS16 rfTS8w4; do
  CMSISDSP_MI355X_LIB=$(lib $v) step 200 python -u bench.py --workload rfft_f32_pscratch --no-cpu-baseline > $O/rf_$v.json 2> $O/rf_$v.err
  show $O/rf_$v.json rfps_$v
done
done
echo all-ok
