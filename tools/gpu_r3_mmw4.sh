#!/bin/bash
# v2 i8 GEMM with 4-wave workgroups (two per CU) against the 8-wave default, alternated; each line
# checks matrix 0 bit-exact.  Output: gpurun_out/mat_var/*.
set -e -o pipefail
for rep in 1 2; do bash tools/run_mat_variants.sh; done
