#!/bin/bash
# Round-3 check H: check G (MFCC paths) + FIR variants (tools/run_fir_variants.sh).
set -e -o pipefail
bash tools/gpu_r3_g.sh
bash tools/run_fir_variants.sh
