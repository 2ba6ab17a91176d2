#!/bin/bash
# Round-5 final check, part 1: the whole -m gpu suite, smoke(), and one bench line per workload
# on the final library (tools/round_lines.sh plus mat_mult_q7 and rfft_f32_pscratch).
set -e -o pipefail
export TMPDIR=/tmp
bash tools/gpu_round_check.sh
bash tools/round_lines.sh r05
O=gpurun_out/lines_r05
for wl in mat_mult_q7 rfft_f32_pscratch mat_mult_fast_q31 fir_q31 fir_fast_q15; do
  timeout -k 10 300 python -u bench.py --workload $wl --no-cpu-baseline > $O/$wl.json 2> $O/$wl.err
  python -c "import json;d=json.load(open('$O/$wl.json'));print('$wl',d['value'],d['unit'],d['roofline'].get('frac'),d['parity'].get('bit_exact'))"
done
echo all-ok
