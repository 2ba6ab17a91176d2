#!/bin/bash
# Round-3 check K: PMC of fir_f32_fma on the default library and the variants (one round name each).
set -e -o pipefail
export TMPDIR=/tmp
bash tools/profile_round.sh r03 fir_f32_fma:hbm
for v in wave nomem; do
  CMSISDSP_MI355X_LIB=$PWD/cmsis-dsp_amd/lib/variants/lib_$v.so bash tools/profile_round.sh r03$v fir_f32_fma:hbm
done
