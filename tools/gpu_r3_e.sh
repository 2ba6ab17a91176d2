#!/bin/bash
# Round-3 check E: MFCC q31/q15 parity through the fused one-launch kernels and, with a
# MI355X_MFCC_FX_FUSED=0 build, through the three-launch path; the mfcc_q31/q15 bench lines;
# the VALU FMA operand-form probe.  Output: gpurun_out/r3e/*.
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3e; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_mfcc_q31.py tests/test_mfcc_q15.py tests/test_pythonwrapper_compat.py \
  -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests_fused.log 2>&1
tail -2 $O/tests_fused.log
CMSISDSP_MI355X_LIB=$PWD/cmsis-dsp_amd/lib/variants/lib_mfcc3.so timeout -k 10 300 python -u -m pytest \
  tests/test_mfcc_q31.py tests/test_mfcc_q15.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/tests_3launch.log 2>&1
tail -2 $O/tests_3launch.log
for wl in mfcc_q31 mfcc_q15; do
  timeout -k 10 200 python -u bench.py --workload $wl --no-cpu-baseline > $O/bench_$wl.json 2> $O/bench_$wl.err
  cat $O/bench_$wl.json
done
timeout -k 10 120 tools/probes/op_rate > $O/op_rate.txt 2>&1
cat $O/op_rate.txt
