#!/bin/bash
# Round-5 GPU step B: PMC profile of mat_mult_q7 (traffic, issue/wait, LDS conflicts, MFMA) and the
# rfft_f32_pscratch mapping sweep (transforms per wave).  Each GPU step has its own time limit.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/b1; mkdir -p $O
step() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step rc=$rc: $*"; exit $rc; }; }
for v in rfT1 rfT4 rfT8; do
  CMSISDSP_MI355X_LIB=cmsis-dsp_amd/lib/variants/lib_$v.so step 200 python -u bench.py --workload rfft_f32_pscratch \
    --no-cpu-baseline > $O/rfps_$v.json 2> $O/rfps_$v.err
  python -c "import json;d=json.load(open('$O/rfps_$v.json'));print('$v',d['value'],d['roofline']['frac'],d['parity']['bit_exact'])"
done
step 200 python -u bench.py --workload rfft_f32_pscratch --no-cpu-baseline > $O/rfps_T2.json 2> $O/rfps_T2.err
python -c "import json;d=json.load(open('$O/rfps_T2.json'));print('T2',d['value'],d['roofline']['frac'],d['parity']['bit_exact'])"
bash tools/profile_round.sh r05b mat_mult_q7:mfma rfft_f32_pscratch:hbm
echo all-ok
