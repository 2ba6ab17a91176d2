#!/bin/bash
# Extra rocprofv3 PMC passes (one counter set per run, each under its own hard limit) of one
# bench workload.  Usage: bash tools/pmc_custom.sh <tag> "<bench args>" "<counters>" ["<counters>" ...]
# Output: gpurun_out/pmcx_<tag>/pass<i>/...
set -o pipefail
TAG=$1; ARGS=$2; shift 2
export TMPDIR=/tmp
O=gpurun_out/pmcx_$TAG; mkdir -p $O
i=0
for C in "$@"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/pass$i -o run -- python -u bench.py $ARGS --no-cpu-baseline \
    > $O/bench$i.json 2> $O/pass$i.err || { echo "pass $i rc=$?"; exit 1; }
  echo "pass $i ok"
done
