#!/bin/bash
# Round-5 GPU step C: A/B of q7 GEMM variants (K step 64 / 128, pinned schedule, no-epilogue
# diagnostic) and the RFFT p-scratch mapping (transforms per wave, waves per workgroup), same box.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/c1; mkdir -p $O
step() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step rc=$rc: $*"; exit $rc; }; }
show() { python -c "import json;d=json.load(open('$1'));print('$2',d['value'],d['roofline']['frac'],d['roofline']['avg_kernel_ms'],d['parity']['bit_exact'])"; }
for rep in 1 2; do
for v in default q7dma q7dmanoepi q7kt128 q7noepi; do
  L=cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so; [ $v = default ] || L=cmsis-dsp_amd/lib/variants/lib_$v.so
  CMSISDSP_MI355X_LIB=$L step 200 python -u bench.py --workload mat_mult_q7 --no-cpu-baseline > $O/q7_$v.json 2> $O/q7_$v.err
  show $O/q7_$v.json q7_$v
done
for v in default rfTS16 rfTS8w4; do
  L=cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so; [ $v = default ] || L=cmsis-dsp_amd/lib/variants/lib_$v.so
  CMSISDSP_MI355X_LIB=$L step 200 python -u bench.py --workload rfft_f32_pscratch --no-cpu-baseline > $O/rf_$v.json 2> $O/rf_$v.err
  show $O/rf_$v.json rfps_$v
done
done
CMSISDSP_MI355X_LIB=cmsis-dsp_amd/lib/variants/lib_q15dma.so step 300 python -u -m pytest tests/test_gpu_rfft_fir_mat.py \
  -k "mat_mult_fixed" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/q15dma_tests.log 2>&1
tail -2 $O/q15dma_tests.log
for v in default q15dma; do
  L=cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so; [ $v = default ] || L=cmsis-dsp_amd/lib/variants/lib_$v.so
  CMSISDSP_MI355X_LIB=$L step 200 python -u bench.py --workload mat_mult_q15 --no-cpu-baseline > $O/q15_$v.json 2> $O/q15_$v.err
  show $O/q15_$v.json q15_$v
done
step 200 python -u bench.py --workload rfft_f32 --no-cpu-baseline > $O/rf_keep.json 2> $O/rf_keep.err
show $O/rf_keep.json rfft_keep_p
echo all-ok
