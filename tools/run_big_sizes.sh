set -e
mkdir -p gpurun_out/big
for n in 512 2048 4096; do
  timeout -k 10 120 python bench.py --workload cfft_f32_1024 --fftlen $n --steps 10 --warmup 3 --no-cpu-baseline --no-companion > gpurun_out/big/cfft_$n.json 2> gpurun_out/big/cfft_$n.err
done
for n in 1024 4096; do
  timeout -k 10 120 python bench.py --workload rfft_f32 --fftlen $n --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/big/rfft_$n.json 2> gpurun_out/big/rfft_$n.err
done
timeout -k 10 120 python bench.py --workload mfcc_f32 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/big/mfcc.json 2> gpurun_out/big/mfcc.err
