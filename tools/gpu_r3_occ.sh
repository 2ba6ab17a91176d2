#!/bin/bash
# Headline kernel occupancy variants (launch-bound waves per SIMD, waves per workgroup) against
# the default build, alternated, each line bit-exact checked.  Output: gpurun_out/occ/*.
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/occ; mkdir -p $O
for rep in 1 2; do
  for L in cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so cmsis-dsp_amd/lib/variants/*.so; do
    v=$(basename $L .so)
    CMSISDSP_MI355X_LIB=$PWD/$L timeout -k 10 200 python -u bench.py --no-companion --no-cpu-baseline > $O/${v}_$rep.json 2> $O/${v}_$rep.err
    python -c "import json;d=json.load(open('$O/${v}_$rep.json'));print('$v',d['value'],d['roofline']['avg_kernel_ms'],d['roofline']['frac'],d['parity']['bit_exact'],d['library'])"
  done
done
