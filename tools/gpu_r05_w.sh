#!/bin/bash
# Round-5 GPU step W: the fused radix-16 inverse with X[N - e] taken from the partner lane by
# ds_bpermute at N <= 1024 (default, MI355X_RFFT_MERGE_XCH=1) against the prefetched second load
# (xch0), and with the registers capped at two waves per SIMD at every N (xw2); RFFT GPU tests on
# every build first, then three alternating inverse timings.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/w1; mkdir -p $O
step() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step rc=$rc: $*"; exit $rc; }; }
lib() { [ $1 = default ] && echo cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so || echo cmsis-dsp_amd/lib/variants/lib_$1.so; }
PT="-x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
for v in default xch0 xw2; do
  CMSISDSP_MI355X_LIB=$(lib $v) step 400 python -u -m pytest tests/test_rfft_fixed.py -m gpu $PT > $O/t_$v.log 2>&1
  echo "$v tests: $(tail -1 $O/t_$v.log)"
done
for rep in 1 2 3; do
for v in default xch0 xw2; do
  CMSISDSP_MI355X_LIB=$(lib $v) step 300 python -u tools/rfft_inv_ab.py 512 1024 2048 4096 > $O/inv_${v}_$rep.txt 2>&1
  grep "^q" $O/inv_${v}_$rep.txt | sed "s/^/$v /"
done
done
echo all-ok
