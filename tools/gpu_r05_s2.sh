#!/bin/bash
# Round-5 GPU step S2: inverse arm_rfft_q31 N = 8192 with the merge fused into the CFFT-4096 kernel
# (s3: half the records -- the tables are symmetric -- and the 4112-slot image in LDS: two workgroups per CU).  The fixed-point RFFT / CFFT / MFCC GPU tests on the new build, then the inverse timing
# (tools/rfft_inv_ab.py 8192 4096) alternating with the two-launch variant (MI355X_RFFT_Q31_INV_FUSED=0).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s3; mkdir -p $O
step() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step rc=$rc: $*"; exit $rc; }; }
lib() { [ $1 = default ] && echo cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so || echo cmsis-dsp_amd/lib/variants/lib_$1.so; }
PT="-x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
step 400 python -u -m pytest tests/test_rfft_fixed.py tests/test_gpu_cfft.py tests/test_mfcc_q15.py -m gpu $PT > $O/t_fused.log 2>&1
echo "fused tests: $(tail -1 $O/t_fused.log)"
for rep in 1 2 3; do
for v in default rfinv31unf; do
  CMSISDSP_MI355X_LIB=$(lib $v) step 300 python -u tools/rfft_inv_ab.py 8192 4096 > $O/inv_${v}_$rep.txt 2>&1
  grep -E "^q" $O/inv_${v}_$rep.txt | sed "s/^/$v /"
done
done
echo all-ok
