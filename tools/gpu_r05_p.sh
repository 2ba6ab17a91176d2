#!/bin/bash
# Round-5 GPU step P: inverse arm_rfft_q31 / q15 fftLenReal 512 .. 4096 with the merge fused into the
# radix-16 CFFT's first pass.  RFFT / MFCC / runtime GPU tests on the new build, then the inverse
# timing (tools/rfft_inv_ab.py) alternating with the two-launch variant (MI355X_RFFT_FX_R16_INV_FUSED=0).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/p1; mkdir -p $O
step() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step rc=$rc: $*"; exit $rc; }; }
lib() { [ $1 = default ] && echo cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so || echo cmsis-dsp_amd/lib/variants/lib_$1.so; }
PT="-x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
step 400 python -u -m pytest tests/test_rfft_fixed.py tests/test_gpu_runtime.py tests/test_mfcc_q31.py tests/test_mfcc_q15.py -m gpu $PT > $O/t_fused.log 2>&1
echo "fused tests: $(tail -1 $O/t_fused.log)"
for rep in 1 2; do
for v in default rfinvunf; do
  CMSISDSP_MI355X_LIB=$(lib $v) step 300 python -u tools/rfft_inv_ab.py > $O/inv_${v}_$rep.txt 2>&1
  sed "s/^/$v /" $O/inv_${v}_$rep.txt
done
done
echo all-ok
