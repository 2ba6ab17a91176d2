#!/bin/bash
# Calibrate the TCC byte counters on a known byte count (cdna_hip_programming.md §7):
# torch's in-place elementwise kernel over 8 GiB reads 8 GiB and writes 8 GiB per pass.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/prof_calib
mkdir -p $OUT
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  name=$(echo $grp | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc_$name -o run -- python tools/hbm_probe.py > $OUT/probe_$name.txt 2> $OUT/pmc_$name.err
done
echo calib done
