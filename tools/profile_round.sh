#!/bin/bash
# rocprofv3 evidence for bench workloads, run on the GPU box (gpurun):
#   * one --kernel-trace --stats pass of the bench command,
#   * separate --pmc passes (never combined with any trace domain; slot limits per pass:
#     SQ <= 8, TCC <= 4 with FETCH_SIZE = 3 and WRITE_SIZE = 2, GRBM <= 2), each under its
#     own hard time limit.
# Usage: bash tools/profile_round.sh <round> <spec>...   spec = name:kind
#   kind = hbm  (traffic + SQ issue counters) | mfma (traffic + SQ + MFMA counters) | trace (trace only)
# The bench arguments of every name are in tools/profile_specs.py.  Output:
# gpurun_out/prof_<round>/<name>/{trace,pmc_*}/..., collected by tools/profile_collect.py.
set -o pipefail
ROUND=$1; shift
export TMPDIR=/tmp
OUT=gpurun_out/prof_$ROUND
mkdir -p $OUT
if [ ! -s $OUT/counters.txt ]; then
  timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
fi
for spec in "$@"; do
  name=${spec%%:*}; kind=${spec##*:}
  args=$(python tools/profile_specs.py $name) || exit 1
  D=$OUT/$name; mkdir -p $D
  BENCH="python -u bench.py $args --no-cpu-baseline"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- $BENCH \
    > $D/bench_trace.json 2> $D/trace.err || { echo "$name trace rc=$?"; exit 1; }
  echo "$name trace ok"
  [ $kind = trace ] && continue
  passes=("FETCH_SIZE" "WRITE_SIZE TCC_EA0_RDREQ_sum"
          "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
          "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE")
  if [ $kind = mfma ]; then
    passes+=("SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE")
  fi
  i=0
  for grp in "${passes[@]}"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $D/pmc_$i -o run -- $BENCH \
      > $D/bench_pmc_$i.json 2> $D/pmc_$i.err
    rc=$?
    if [ $rc -ne 0 ]; then
      echo "$name pmc pass $i ($grp) rc=$rc"; tail -3 $D/pmc_$i.err
      # a time limit / kill (possible counter hang) ends the script; an early error of the
      # optional MFMA pass (a counter this ROCm does not expose) does not
      if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $i -le 4 ]; then exit $rc; fi
    fi
  done
  echo "$name pmc ok"
done
