#!/bin/bash
# rocprofv3 kernel trace (+ --stats) of tools/bench_filters.py workloads on the GPU box, and
# one FETCH_SIZE / WRITE_SIZE pass each (separate runs, own time limits).
# Usage: bash tools/profile_filters.sh <tag> <workload>...  -> gpurun_out/prof_filters_<tag>/<workload>/
set -o pipefail
TAG=$1; shift
export TMPDIR=/tmp
for w in "$@"; do
  D=gpurun_out/prof_filters_$TAG/$w; mkdir -p $D
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- \
    python -u tools/bench_filters.py $w > $D/bench.json 2> $D/trace.err || { echo "$w trace rc=$?"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/pmc_1 -o run -- \
    python -u tools/bench_filters.py $w > $D/bench_pmc_1.json 2> $D/pmc_1.err || { echo "$w pmc1 rc=$?"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/pmc_2 -o run -- \
    python -u tools/bench_filters.py $w > $D/bench_pmc_2.json 2> $D/pmc_2.err || { echo "$w pmc2 rc=$?"; exit 1; }
  echo "$w ok: $(cat $D/bench.json)"
done
