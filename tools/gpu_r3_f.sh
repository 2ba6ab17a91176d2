#!/bin/bash
# Round-3 check F: rocprofv3 trace + PMC of the fused MFCC q31 / q15 kernels.
set -e -o pipefail
export TMPDIR=/tmp
bash tools/profile_round.sh r03 mfcc_q31:hbm mfcc_q15:hbm
