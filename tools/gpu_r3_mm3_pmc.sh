#!/bin/bash
# PMC passes (one counter group per run, each under its own hard limit) of the i8 GEMM v3 for
# mat_mult_q15.  Output: gpurun_out/mm3pmc/pmc_<i>/...
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/mm3pmc; mkdir -p $O
W=${1:-mat_mult_q15}
i=0
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" \
         "GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum" \
         "SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_VMEM SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_WAVES"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/pmc_$i -o run -- python -u bench.py --workload $W --steps 4 --warmup 1 --no-cpu-baseline \
    > $O/bench$i.json 2> $O/pass$i.err || { echo "pass $i rc=$?"; exit 1; }
  echo "pass $i ok"
done
python3 tools/pmc_summary.py $O i8v3 > $O/summary.txt 2>&1; cat $O/summary.txt | head -60
