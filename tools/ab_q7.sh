#!/bin/bash
# Same-box A/B of mat_mult_q7 build variants (tools/build_variant.sh): bench lines alternating,
# default library and each variant in turn.  Usage: tools/ab_q7.sh <outdir> <reps> variant...
OUT=$1; REPS=$2; shift 2
mkdir -p $OUT
for rep in $(seq 1 $REPS); do
  for v in default "$@"; do
    if [ $v = default ]; then
      timeout -k 10 120 python bench.py --workload mat_mult_q7 --steps 10 --warmup 3 > $OUT/$v.$rep.json 2>/dev/null || exit 1
    else
      CMSISDSP_MI355X_LIB=cmsis-dsp_amd/lib/variants/lib_$v.so timeout -k 10 120 python bench.py --workload mat_mult_q7 --steps 10 --warmup 3 > $OUT/$v.$rep.json 2>/dev/null || exit 1
    fi
  done
done
