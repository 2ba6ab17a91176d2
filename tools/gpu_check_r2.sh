#!/bin/bash
# Round-2 GPU confirmation on one MI355X: the whole -m gpu suite, smoke(), the default
# bench line (configs[1] + configs[3] strong scaling), a 2-rank rehearsal of --gpus 2 on
# the one device (gloo: RCCL needs one GPU per rank), and the mat_mult_f32 line.
# Every GPU step has its own time limit; a test FAILURE (pytest rc 1) still lets the
# bench run, anything else (fault, abort, timeout) ends the script.
# Output: gpurun_out/$OUT/*.
OUT=${1:-r2}
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/$OUT
rc=0
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/$OUT/gpu_tests.log 2>&1 || rc=$?
tail -5 gpurun_out/$OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$OUT/smoke.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > gpurun_out/$OUT/bench_default.json 2> gpurun_out/$OUT/bench_default.err || exit $?
cat gpurun_out/$OUT/bench_default.json
timeout -k 10 300 python -u bench.py --gpus 2 --no-cpu-baseline > gpurun_out/$OUT/bench_gpus2.json \
  2> gpurun_out/$OUT/bench_gpus2.err || exit $?
cat gpurun_out/$OUT/bench_gpus2.json
timeout -k 10 200 python -u bench.py --workload mat_mult_f32 --steps 5 --warmup 2 \
  > gpurun_out/$OUT/bench_mat_mult_f32.json 2> gpurun_out/$OUT/bench_mat_mult_f32.err || exit $?
cat gpurun_out/$OUT/bench_mat_mult_f32.json
exit $rc
