#!/bin/bash
# configs[3] q31 residency variants (LDS slots -> 2 workgroups per CU; stage-3/4 twiddles in LDS;
# 4 waves per SIMD) against the default build, alternated; config3 lines are bit-exact checked.
# Output: gpurun_out/fxocc/*.
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/fxocc; mkdir -p $O
for rep in 1 2; do
  for L in cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so cmsis-dsp_amd/lib/variants/*.so; do
    v=$(basename $L .so)
    CMSISDSP_MI355X_LIB=$PWD/$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > $O/${v}_$rep.json 2> $O/${v}_$rep.err
    python -c "import json;d=json.load(open('$O/${v}_$rep.json'));c=d['config3'];print('$v',d['value'],*[(k,c[k]['value'],c[k]['roofline']['frac'],c[k]['parity']['bit_exact']) for k in ('q31','q15')])"
  done
done
