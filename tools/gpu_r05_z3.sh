#!/bin/bash
# Round-5 final confirmation on the final library: the whole -m gpu suite, smoke(), the default
# bench line (+ f32 2048 / 4096), the mat_mult_q7 line and its profile (the q7 default changed).
set -e -o pipefail
export TMPDIR=/tmp
bash tools/gpu_round_check.sh
mkdir -p gpurun_out/rc
timeout -k 10 300 python -u bench.py --workload mat_mult_q7 > gpurun_out/rc/mat_mult_q7.json 2> gpurun_out/rc/mat_mult_q7.err
cat gpurun_out/rc/mat_mult_q7.json
rm -rf gpurun_out/prof_r05
bash tools/profile_round.sh r05 mat_mult_q7:mfma
echo all-ok
