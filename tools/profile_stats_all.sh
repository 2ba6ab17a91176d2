#!/bin/bash
# rocprofv3 kernel-trace statistics for every bench workload (one short bench run each),
# plus the f32 CFFT specialists at N=2048/4096.
# Output: gpurun_out/stats/<workload>/run_kernel_stats.csv (+ the bench JSON line).
set -e -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/stats
for wl in cfft_f32_1024 cfft_q31_4096 cfft_q15_4096 rfft_f32 rfft_q31 rfft_q15 fir_f32 fir_q15 fir_q31 \
          fir_fast_q15 fir_fast_q31 conv_f32 mat_mult_f32 mat_mult_q15 mat_mult_q31 mat_mult_fast_q31 mfcc_f32; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stats/$wl -o run -- \
    python bench.py --workload $wl --steps 10 --warmup 3 --no-companion --no-cpu-baseline \
    > gpurun_out/stats/$wl.json 2> gpurun_out/stats/$wl.err
  echo "$wl done"
done
for n in 2048 4096; do
  wl=cfft_f32_$n
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stats/$wl -o run -- \
    python bench.py --fftlen $n --steps 10 --warmup 3 --no-companion --no-cpu-baseline \
    > gpurun_out/stats/$wl.json 2> gpurun_out/stats/$wl.err
  echo "$wl done"
done
