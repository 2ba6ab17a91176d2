#!/bin/bash
# Round-3 final bench lines of every workload (default line with cpu_baseline + the others),
# each under its own limit; stops at the first failure.  Output: gpurun_out/r3lines/*.
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3lines; mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err
for wl in fir_f32 fir_f32_fma fir_q15 mfcc_f32 mfcc_q31 mfcc_q15 rfft_f32 rfft_q31 rfft_q15 conv_f32 mat_mult_f32 mat_mult_q15 mat_mult_q31; do
  timeout -k 10 200 python -u bench.py --workload $wl --no-cpu-baseline > $O/$wl.json 2> $O/$wl.err
  python -c "import json;d=json.load(open('$O/$wl.json'));print('$wl',d['value'],d['unit'],d['roofline'].get('frac'),d['parity'].get('bit_exact'))"
done
