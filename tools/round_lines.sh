#!/bin/bash
# Bench lines of every workload on the current code (one box), each under its own limit; stops
# at the first failure.  The default line and the BASELINE configs (fir_f32 = configs[2],
# mat_mult_f32 = configs[4]) carry cpu_baseline; the other workloads skip it to save box time.
# Usage: bash tools/round_lines.sh <tag>     Output: gpurun_out/lines_<tag>/*.
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/lines_${1:-cur}; mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err
for wl in fir_f32 mat_mult_f32 fir_f32_fma fir_q15 fir_q31 fir_fast_q15 fir_fast_q31 mfcc_f32 mfcc_q31 mfcc_q15 rfft_f32 rfft_f32_pscratch rfft_q31 rfft_q15 conv_f32 mat_mult_q7 mat_mult_q15 mat_mult_q31 mat_mult_fast_q31; do
  cb="--no-cpu-baseline"
  case $wl in fir_f32|mat_mult_f32) cb="";; esac
  timeout -k 10 300 python -u bench.py --workload $wl $cb > $O/$wl.json 2> $O/$wl.err
  python -c "import json;d=json.load(open('$O/$wl.json'));print('$wl',d['value'],d['unit'],d['roofline'].get('frac'),d['parity'].get('bit_exact'),(d.get('cpu_baseline') or {}).get('value'))"
done
timeout -k 10 200 python -u tools/bench_filters.py fir_q7 > $O/fir_q7.json 2> $O/fir_q7.err
python -c "import json;d=json.loads(open('$O/fir_q7.json').read().splitlines()[0]);print('fir_q7',d['input_gsamples_per_s'],d['bit_exact'])"
