#!/bin/bash
# Run on the GPU box (gpurun): rocprofv3 kernel-trace/stats and PMC passes for one bench
# workload.  Counters are collected in separate passes (one TCC byte counter per pass;
# never combined with sys/runtime tracing).  Output: gpurun_out/prof_<tag>/...
# Usage: bash tools/profile_pmc.sh <workload> <tag> [extra bench args]
set -e
WL=${1:-cfft_f32_1024}; TAG=${2:-$WL}; shift 2 || true
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
BENCH="python bench.py --workload $WL --steps 5 --warmup 2 --no-companion --no-cpu-baseline $@"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $BENCH > $OUT/bench_trace.json 2> $OUT/trace.err
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE"; do
  name=$(echo $grp | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc_$name -o run -- $BENCH > $OUT/bench_$name.json 2> $OUT/pmc_$name.err
done
echo "profile $TAG done"
