#!/bin/bash
# Round-3 closing check on one MI355X: the whole -m gpu suite, smoke(), the default bench line,
# the default line through a one-rank RCCL group, and the mfcc_f32 kernel trace + PMC traffic of
# the regrouped Mel stage.  Every GPU step has its own limit; stops at the first failure.
# Output: gpurun_out/final/*.
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/final; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/gpu_tests.log 2>&1
tail -2 $O/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err
cat $O/bench_default.json
CMSISDSP_DIST_SINGLE=1 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29611 \
  timeout -k 10 300 python -u bench.py --gpus 1 --scatter > $O/bench_rccl1.json 2> $O/bench_rccl1.err
cat $O/bench_rccl1.json
bash tools/profile_round.sh r03 cfft_q31_4096_strong1M:hbm > $O/profile.log 2>&1
tail -3 $O/profile.log
