#!/bin/bash
# Round-3 check J: FIR f32 variants (bench lines) + PMC of the default fir_f32 / fir_f32_fma.
set -e -o pipefail
export TMPDIR=/tmp
bash tools/run_fir_variants.sh
bash tools/profile_round.sh r03 fir_f32:hbm fir_f32_fma:hbm
