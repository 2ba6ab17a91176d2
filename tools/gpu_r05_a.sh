#!/bin/bash
# Round-5 GPU check A: the new -m gpu tests (per-thread resource release, q7 GEMM, RFFT p
# pinning / P_SCRATCH), the MFCC fixed-point tests on the one-launch variant build (the mvals
# race fix), the mat_mult_q7 and rfft_f32_pscratch bench lines and a kernel trace of each.
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/a1; mkdir -p $O
step() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step rc=$rc: $*"; exit $rc; }; }
step 400 python -u -m pytest tests/test_gpu_runtime.py tests/test_gpu_rfft_fir_mat.py -k "q7 or short_lived or release_thread or rfft" \
  -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
tail -3 $O/tests.log
CMSISDSP_MI355X_LIB=cmsis-dsp_amd/lib/variants/lib_mfcc1l.so step 300 python -u -m pytest tests/test_mfcc_q31.py \
  tests/test_mfcc_q15.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/mfcc1l.log 2>&1
tail -2 $O/mfcc1l.log
step 200 python -u bench.py --workload mat_mult_q7 > $O/q7.json 2> $O/q7.err
cat $O/q7.json
CMSISDSP_MI355X_LIB=cmsis-dsp_amd/lib/variants/lib_q7s.so step 200 python -u bench.py --workload mat_mult_q7 \
  --no-cpu-baseline > $O/q7s.json 2> $O/q7s.err
cat $O/q7s.json
for v in i8pin6 i8pin10; do
  CMSISDSP_MI355X_LIB=cmsis-dsp_amd/lib/variants/lib_$v.so step 200 python -u bench.py --workload mat_mult_q15 \
    --no-cpu-baseline > $O/q15_$v.json 2> $O/q15_$v.err
  cat $O/q15_$v.json
done
step 200 python -u bench.py --workload mat_mult_q15 --no-cpu-baseline > $O/q15.json 2> $O/q15.err
cat $O/q15.json
step 200 python -u bench.py --workload rfft_f32_pscratch > $O/rfps.json 2> $O/rfps.err
cat $O/rfps.json
step 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_q7 -o run -- python -u bench.py \
  --workload mat_mult_q7 --steps 10 --warmup 3 --no-cpu-baseline > $O/q7_trace.json 2>&1
step 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_rfps -o run -- python -u bench.py \
  --workload rfft_f32_pscratch --steps 10 --warmup 3 --no-cpu-baseline > $O/rfps_trace.json 2>&1
echo all-ok
