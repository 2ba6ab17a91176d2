#!/bin/bash
# Round-3 i8 GEMM v3 (packed planes + LDS-DMA GEMM): mat_mult parity, bench lines of the default
# library and its variants, kernel trace of both workloads.  Each GPU step has its own limit;
# stops at the first failure.  Output: gpurun_out/mm3/*.
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/mm3; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "mat_mult" --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/tests.log 2>&1
tail -2 $O/tests.log
bash tools/run_mat_variants.sh
for w in mat_mult_q15 mat_mult_q31; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$w -o run -- \
    python3 bench.py --workload $w --steps 6 --warmup 2 --no-cpu-baseline > $O/prof_$w.log 2>&1
done
find $O -name "*kernel_stats.csv" | while read f; do echo "== $f"; cut -d, -f1-5 "$f" | grep -i "mi355x\|Name" | head -8; done
