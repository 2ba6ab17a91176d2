#!/bin/bash
# Round-3 check M: the default bench line (configs[1] + config3 + cpu_baseline), bench lines of
# the other workloads, and r03 profiles of the headline / configs[3] / mfcc_f32 / rfft_f32 / mat_mult_f32.
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3m; mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err
cat $O/bench_default.json | head -c 600; echo
for wl in fir_f32 fir_f32_fma fir_q15 mfcc_f32 mfcc_q31 mfcc_q15 rfft_f32 rfft_q31 rfft_q15 conv_f32 mat_mult_f32 mat_mult_q15 mat_mult_q31; do
  timeout -k 10 200 python -u bench.py --workload $wl --no-cpu-baseline > $O/$wl.json 2> $O/$wl.err
  python -c "import json;d=json.load(open('$O/$wl.json'));print('$wl',d['value'],d['unit'],d['roofline'].get('frac'),d['roofline'].get('avg_kernel_ms'),d['parity'].get('bit_exact'))"
done
bash tools/profile_round.sh r03 cfft_f32_1024:hbm cfft_q31_4096_strong1M:hbm cfft_q15_4096_strong1M:hbm mfcc_f32:hbm rfft_f32:hbm mat_mult_f32:mfma
