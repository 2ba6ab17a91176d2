#!/bin/bash
# Round-5 final confirmation on the final library: the whole -m gpu suite, smoke(), the default
# bench line (+ f32 2048 / 4096), then rocprofv3 evidence for the radix-16 fused RFFT (fftLenReal 1024).
set -e -o pipefail
export TMPDIR=/tmp
rm -rf gpurun_out/rc gpurun_out/prof_r05
bash tools/gpu_round_check.sh
bash tools/profile_round.sh r05 rfft_q31_1024:hbm rfft_q15_1024:hbm
echo all-ok
