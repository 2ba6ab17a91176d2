#!/bin/bash
# Round-5 final confirmation (after the fused inverse RFFTs): the whole -m gpu suite, smoke(), the
# default bench line (+ f32 2048 / 4096), every workload's line, the radix-16 fused RFFT profiles.
set -e -o pipefail
export TMPDIR=/tmp
rm -rf gpurun_out/rc gpurun_out/prof_r05 gpurun_out/lines_r05final
bash tools/gpu_round_check.sh
bash tools/round_lines.sh r05final
bash tools/profile_round.sh r05 rfft_q31_1024:hbm rfft_q15_1024:hbm
echo all-ok
