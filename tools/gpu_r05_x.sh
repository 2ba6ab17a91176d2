#!/bin/bash
# Round-5 GPU step X: the fused radix-16 inverse at fftLenReal 4096 (P = 128 lanes per transform) with
# X[N - e] through the transform's LDS image (MI355X_RFFT_MERGE_LDSX=1) against the second set of
# loads (default); RFFT GPU tests on the variant first, then three alternating inverse timings.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/x1; mkdir -p $O
step() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step rc=$rc: $*"; exit $rc; }; }
lib() { [ $1 = default ] && echo cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so || echo cmsis-dsp_amd/lib/variants/lib_$1.so; }
PT="-x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
CMSISDSP_MI355X_LIB=$(lib ldsx1) step 400 python -u -m pytest tests/test_rfft_fixed.py -m gpu $PT > $O/t_ldsx1.log 2>&1
echo "ldsx1 tests: $(tail -1 $O/t_ldsx1.log)"
for rep in 1 2 3; do
for v in default ldsx1; do
  CMSISDSP_MI355X_LIB=$(lib $v) step 300 python -u tools/rfft_inv_ab.py 4096 > $O/inv_${v}_$rep.txt 2>&1
  grep "^q" $O/inv_${v}_$rep.txt | sed "s/^/$v /"
done
done
echo all-ok
