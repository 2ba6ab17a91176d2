#!/bin/bash
# MFCC q31 / q15 on one MI355X: the GPU parity tests (fixed-point MFCC, fixed-point RFFT, the
# cmsisdsp wrapper replays), then one bench line per workload.  Output: gpurun_out/mfx/*.
set -o pipefail
mkdir -p gpurun_out/mfx
timeout -k 10 300 python -u -m pytest tests/test_mfcc_q15.py tests/test_mfcc_q31.py tests/test_rfft_fixed.py tests/test_pythonwrapper_compat.py \
  -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/mfx/tests.log 2>&1
rc=$?; tail -3 gpurun_out/mfx/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for w in ${WORKLOADS:-mfcc_q15 mfcc_q31}; do
  timeout -k 10 200 python -u bench.py --workload $w --steps 10 --warmup 3 > gpurun_out/mfx/$w.json \
    2> gpurun_out/mfx/$w.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/mfx/$w.json'));print('$w',d['value'],d['roofline']['frac'],d['parity'],d.get('cpu_baseline',{}).get('value'))"
done
