#!/bin/bash
# Round-3 check I: full -m gpu suite, MFCC schedules (check G), MFCC q31/q15 profiles.
set -e -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r3/gpu_tests.log 2>&1
tail -2 gpurun_out/r3/gpu_tests.log
bash tools/gpu_r3_g.sh
bash tools/profile_round.sh r03 mfcc_q31:hbm mfcc_q15:hbm
