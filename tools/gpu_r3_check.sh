#!/bin/bash
# Round-3 GPU check: the -m gpu suite (new long-FIR / cache / ordering tests first, then
# everything) and the fir_f32 bench line.  Each GPU step has its own time limit; the script
# stops at the first failure.  Output: gpurun_out/r3/*.
set -e -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3
timeout -k 10 300 python -u -m pytest tests/test_fir_long.py tests/test_gpu_runtime.py -m gpu -x -v \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3/gpu_new.log 2>&1
tail -3 gpurun_out/r3/gpu_new.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r3/gpu_tests.log 2>&1
tail -3 gpurun_out/r3/gpu_tests.log
timeout -k 10 200 python -u bench.py --workload fir_f32 --no-cpu-baseline > gpurun_out/r3/bench_fir.json 2> gpurun_out/r3/bench_fir.err
cat gpurun_out/r3/bench_fir.json
