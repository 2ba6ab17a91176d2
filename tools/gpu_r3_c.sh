#!/bin/bash
# Round-3 check C: mat_mult q15/q31 parity with the swizzled LDS planes, then rocprofv3 traces and
# PMC passes of fir_f32, fir_f32_fma, mat_mult_q15 and mat_mult_q31.  Output: gpurun_out/r3c,
# gpurun_out/prof_r03/*.
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3c; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "mat_mult" --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/tests.log 2>&1
tail -2 $O/tests.log
bash tools/profile_round.sh r03 fir_f32:hbm fir_f32_fma:hbm mat_mult_q15:mfma mat_mult_q31:mfma
