#!/bin/bash
# Round-5 final check, part 2: rocprofv3 kernel traces + PMC passes of the headline, configs[3],
# configs[4] and the i8 GEMMs on the final library (tools/profile_round.sh).
set -o pipefail
export TMPDIR=/tmp
bash tools/profile_round.sh r05 cfft_f32_1024:hbm mat_mult_f32:mfma mat_mult_q7:mfma mat_mult_q15:mfma \
  mat_mult_q31:mfma rfft_f32_pscratch:hbm cfft_q15_4096_strong1M:hbm cfft_q31_4096_strong1M:hbm && echo all-ok
