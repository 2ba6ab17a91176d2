#!/bin/bash
# Round-3 check L: full -m gpu suite, then fir_f32 / fir_f32_fma profiles (trace + PMC).
set -e -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r3/gpu_tests.log 2>&1
tail -2 gpurun_out/r3/gpu_tests.log
bash tools/profile_round.sh r03 fir_f32:hbm fir_f32_fma:hbm
