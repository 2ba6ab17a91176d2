set -e
mkdir -p gpurun_out/sizes2
for wl in cfft_f32_1024 cfft_q31_4096 cfft_q15_4096; do
  for n in 16 32 64 128 256 512; do
    timeout -k 10 120 python bench.py --workload $wl --fftlen $n --steps 10 --warmup 3 --no-cpu-baseline --no-companion \
      > gpurun_out/sizes2/${wl}_$n.json 2> gpurun_out/sizes2/${wl}_$n.err
  done
done
