#!/bin/bash
# Round-5 GPU step H: the 2-wave latency-shaped N = 1024 drop-in kernel — drop-in / runtime /
# example tests on it, then per-call latency against the one-wave kernel (lat0), same box.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/h1; mkdir -p $O
step() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step rc=$rc: $*"; exit $rc; }; }
PT="-x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
step 400 python -u -m pytest tests/test_gpu_cfft.py tests/test_examples.py tests/test_gpu_runtime.py -m gpu $PT > $O/tests.log 2>&1
echo "tests: $(tail -1 $O/tests.log)"
L=cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so; L0=cmsis-dsp_amd/lib/variants/lib_lat0.so; R=oracle/_ref/libcmsisdsp_ref.so
for rep in 1 2 3; do
  step 120 tools/latency/dropin_latency $L $R 2000 > $O/lat1_$rep.json; echo "lat1 $(cat $O/lat1_$rep.json)"
  step 120 tools/latency/dropin_latency $L0 $R 2000 > $O/lat0_$rep.json; echo "lat0 $(cat $O/lat0_$rep.json)"
done
step 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- tools/latency/dropin_latency $L $R 500 > $O/prof_lat1.json 2>&1
echo all-ok
