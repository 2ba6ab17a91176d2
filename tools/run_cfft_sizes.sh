# Throughput of every f32 / q31 / q15 CFFT length (generic kernels + specialists), same
# bytes per launch as the headline configs.  Output: gpurun_out/sizes/*.json
set -e
mkdir -p gpurun_out/sizes
for wl in cfft_f32_1024 cfft_q31_4096 cfft_q15_4096; do
  for n in 16 32 64 128 256 512 1024 2048 4096; do
    timeout -k 10 120 python bench.py --workload $wl --fftlen $n --steps 10 --warmup 3 --no-cpu-baseline --no-companion \
      > gpurun_out/sizes/${wl%%_*}_${wl#*_}_$n.json 2> gpurun_out/sizes/${wl}_$n.err
  done
done
