#!/bin/bash
# Round-5 GPU step E: bit-exact tests then A/B of the two-workgroups-per-CU LDS-DMA GEMMs (q7, q15)
# and the one-launch MFCC at 3 waves/SIMD (twiddles re-read per group), same box.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/e1; mkdir -p $O
step() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step rc=$rc: $*"; exit $rc; }; }
show() { python -c "import json;d=json.load(open('$1'));p=d['parity'];print('$2',d['value'],d['roofline']['frac'],d['roofline']['avg_kernel_ms'],p.get('bit_exact',p) if isinstance(p,dict) else p)"; }
lib() { [ $1 = default ] && echo cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so || echo cmsis-dsp_amd/lib/variants/lib_$1.so; }
PT="-x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
for v in q7dma1 q7dma2; do
  CMSISDSP_MI355X_LIB=$(lib $v) step 300 python -u -m pytest tests/test_gpu_rfft_fir_mat.py tests/test_gpu_runtime.py -k q7 $PT > $O/t_$v.log 2>&1
  echo "$v: $(tail -1 $O/t_$v.log)"
done
CMSISDSP_MI355X_LIB=$(lib q15dma2) step 300 python -u -m pytest tests/test_gpu_rfft_fir_mat.py -k "mat_mult_fixed or mat_mult_fast" $PT > $O/t_q15dma2.log 2>&1
echo "q15dma2: $(tail -1 $O/t_q15dma2.log)"
for v in mfcc1lwg3 mfcc1ltw3; do
  CMSISDSP_MI355X_LIB=$(lib $v) step 300 python -u -m pytest tests/test_mfcc_q31.py tests/test_mfcc_q15.py -m gpu $PT > $O/t_$v.log 2>&1
  echo "$v: $(tail -1 $O/t_$v.log)"
done
for rep in 1 2; do
for v in default q7dma1 q7dma2; do
  CMSISDSP_MI355X_LIB=$(lib $v) step 200 python -u bench.py --workload mat_mult_q7 --no-cpu-baseline > $O/q7_$v.json 2> $O/q7_$v.err
  show $O/q7_$v.json q7_$v
done
for v in default q15dma2; do
  CMSISDSP_MI355X_LIB=$(lib $v) step 200 python -u bench.py --workload mat_mult_q15 --no-cpu-baseline > $O/q15_$v.json 2> $O/q15_$v.err
  show $O/q15_$v.json q15_$v
done
for w in mfcc_q31 mfcc_q15; do
for v in default mfcc1l mfcc1lwg3 mfcc1ltw3 mfcc1ltw; do
  CMSISDSP_MI355X_LIB=$(lib $v) step 200 python -u bench.py --workload $w --no-cpu-baseline > $O/${w}_$v.json 2> $O/${w}_$v.err
  show $O/${w}_$v.json ${w}_$v
done
done
for v in default f32x1; do
  CMSISDSP_MI355X_LIB=$(lib $v) step 200 python -u bench.py --workload mat_mult_f32 --no-cpu-baseline > $O/f32_$v.json 2> $O/f32_$v.err
  python -c "import json;d=json.load(open('$O/f32_$v.json'));print('f32_$v',d['value'],d['roofline']['frac'],d['roofline']['avg_kernel_ms'],d['parity']['fmaf_chain_bit_exact'])"
done
done
echo all-ok
