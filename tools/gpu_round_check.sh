#!/bin/bash
# Round-end GPU confirmation on one MI355X: the whole -m gpu suite, smoke(), the default
# bench line and the f32 N=2048/4096 specialist bench lines.  Every GPU step has its own
# time limit and the script stops at the first failure.
# Output: gpurun_out/rc/*.
set -e -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/rc
timeout -k 10 780 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/rc/gpu_tests.log 2>&1
tail -3 gpurun_out/rc/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
  > gpurun_out/rc/smoke.log 2>&1
timeout -k 10 200 python -u bench.py > gpurun_out/rc/bench_default.json 2> gpurun_out/rc/bench_default.err
cat gpurun_out/rc/bench_default.json
for n in 2048 4096; do
  timeout -k 10 120 python -u bench.py --fftlen $n --no-companion --no-cpu-baseline \
    > gpurun_out/rc/bench_f32_$n.json 2> gpurun_out/rc/bench_f32_$n.err
  cat gpurun_out/rc/bench_f32_$n.json
done
