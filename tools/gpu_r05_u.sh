#!/bin/bash
# Round-5 GPU step U: the fused radix-16 inverse with its register allocation capped at two waves
# per SIMD (MI355X_RFFT_MERGE_WAVES=2: q31 fftLenReal 512 / 2048 then spill 12 / 60 VGPRs instead of
# running at one wave) against the default; RFFT GPU tests on the variant first.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/u1; mkdir -p $O
step() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step rc=$rc: $*"; exit $rc; }; }
lib() { [ $1 = default ] && echo cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so || echo cmsis-dsp_amd/lib/variants/lib_$1.so; }
PT="-x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
CMSISDSP_MI355X_LIB=$(lib rmw2) step 400 python -u -m pytest tests/test_rfft_fixed.py -m gpu $PT > $O/t_rmw2.log 2>&1
echo "rmw2 tests: $(tail -1 $O/t_rmw2.log)"
for rep in 1 2 3; do
for v in default rmw2; do
  CMSISDSP_MI355X_LIB=$(lib $v) step 300 python -u tools/rfft_inv_ab.py 512 2048 > $O/inv_${v}_$rep.txt 2>&1
  grep -E "^q31" $O/inv_${v}_$rep.txt | sed "s/^/$v /"
done
done
echo all-ok
