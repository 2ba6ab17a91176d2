#!/bin/bash
# Headline kernel with 16-B loads + permlane32 swap: swap semantics probe, CFFT/RFFT GPU parity,
# then the headline bench line of the new library and of the 8-B-load build (lib_ld8), alternated.
# Output: gpurun_out/ld16/*.
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ld16; mkdir -p $O
timeout -k 10 60 ./tools/probes/permlane32_swap > $O/swap_probe.txt 2>&1
cat $O/swap_probe.txt
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "cfft or rfft or mfcc or example or smoke or runtime" --timeout 120 \
  --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
tail -2 $O/tests.log
for rep in 1 2 3; do
  for L in cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so cmsis-dsp_amd/lib/variants/lib_ld8.so; do
    v=$(basename $L .so)
    CMSISDSP_MI355X_LIB=$PWD/$L timeout -k 10 200 python -u bench.py --no-companion --no-cpu-baseline > $O/${v}_$rep.json 2> $O/${v}_$rep.err
    python -c "import json;d=json.load(open('$O/${v}_$rep.json'));print('$v',d['value'],d['roofline']['avg_kernel_ms'],d['roofline']['frac'],d['parity']['bit_exact'])"
  done
done
