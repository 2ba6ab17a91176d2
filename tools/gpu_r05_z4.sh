#!/bin/bash
# Round-5 confirmation after the fused N=8192 forward RFFT q31/q15: the whole -m gpu suite,
# smoke(), the default bench line (+ f32 2048 / 4096), the rfft_q31 / rfft_q15 lines and their
# profiles (trace + HBM traffic).
set -e -o pipefail
export TMPDIR=/tmp
bash tools/gpu_round_check.sh
for w in rfft_q31 rfft_q15; do
  timeout -k 10 200 python -u bench.py --workload $w > gpurun_out/rc/$w.json 2> gpurun_out/rc/$w.err
  cat gpurun_out/rc/$w.json
done
rm -rf gpurun_out/prof_r05
bash tools/profile_round.sh r05 rfft_q31:hbm rfft_q15:hbm
echo all-ok
