#!/bin/bash
# Round-3 check B: MFCC f32 bit-exact on the GPU, the mfcc_f32 / mfcc_q31 bench lines, and a
# 2-rank rehearsal of --scatter + the N>1 cpu_baseline on the one-GPU box (gloo, both ranks on
# GPU 0, a 64K global batch).  Output: gpurun_out/r3b/*.
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3b; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_mfcc.py tests/test_pythonwrapper_compat.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gpu_mfcc.log 2>&1
tail -2 $O/gpu_mfcc.log
timeout -k 10 200 python -u bench.py --workload mfcc_f32 --no-cpu-baseline > $O/bench_mfcc_f32.json 2> $O/bench_mfcc_f32.err
cat $O/bench_mfcc_f32.json
timeout -k 10 200 python -u bench.py --workload mfcc_q31 --no-cpu-baseline > $O/bench_mfcc_q31.json 2> $O/bench_mfcc_q31.err
cat $O/bench_mfcc_q31.json
timeout -k 10 400 python -u bench.py --gpus 2 --global-batch 65536 --scatter --steps 5 --warmup 2 --cpu-secs 0.5 \
  > $O/bench_gpus2_scatter.json 2> $O/bench_gpus2_scatter.err
cat $O/bench_gpus2_scatter.json
