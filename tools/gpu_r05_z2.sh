#!/bin/bash
# Round-5 final check, part 2: rocprofv3 kernel traces + PMC passes of the headline, configs[3],
# configs[4] and the i8 GEMMs on the final library (tools/profile_round.sh).
set -o pipefail
export TMPDIR=/tmp
bash tools/profile_round.sh r05 cfft_f32_1024:hbm mat_mult_f32:mfma mat_mult_q7:mfma mat_mult_q15:mfma \
  mat_mult_q31:mfma rfft_f32_pscratch:hbm cfft_q15_4096_strong1M:hbm cfft_q31_4096_strong1M:hbm && echo all-ok
# q7: the pinned steady-step order (MI355X_Q7_SCHED=1) against the default, after its tests
O=gpurun_out/z2ab; mkdir -p $O
L=cmsis-dsp_amd/lib/variants/lib_q7sched.so
CMSISDSP_MI355X_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_rfft_fir_mat.py tests/test_gpu_runtime.py -k q7 \
  -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/t_q7sched.log 2>&1 || { echo "q7sched tests failed"; exit 1; }
echo "q7sched tests: $(tail -1 $O/t_q7sched.log)"
for rep in 1 2 3; do
  for v in default q7sched; do
    LL=cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so; [ $v = default ] || LL=$L
    CMSISDSP_MI355X_LIB=$LL timeout -k 10 200 python -u bench.py --workload mat_mult_q7 --no-cpu-baseline > $O/q7_$v.json 2> $O/q7_$v.err || exit 1
    python -c "import json;d=json.load(open('$O/q7_$v.json'));print('q7_$v',d['value'],d['roofline']['frac'],d['parity']['bit_exact'])"
  done
done
