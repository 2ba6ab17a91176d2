#!/bin/bash
# Timing probes of the i8 GEMM v3 K loop (probe builds: results are wrong by design) plus the
# default library.  Output: gpurun_out/mm3probe/*.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/mm3probe; mkdir -p $O
for L in cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so cmsis-dsp_amd/lib/variants/*.so; do
  v=$(basename $L .so)
  CMSISDSP_MI355X_LIB=$PWD/$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- \
    python3 bench.py --workload mat_mult_q15 --steps 4 --warmup 1 --no-cpu-baseline > $O/$v.json 2> $O/$v.err || exit 1
  grep -h "i8v3" $O/$v/run_kernel_stats.csv | awk -F, -v v=$v '{print v, $4, $5}'
done
