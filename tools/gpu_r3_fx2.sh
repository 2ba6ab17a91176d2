#!/bin/bash
# q31 N=4096 at two workgroups per CU: fixed-point CFFT / RFFT / MFCC parity, then the rfft_q31 and
# mfcc_q31 bench lines (which reuse the CFFT kernels) for the new build and the previous one.
# Output: gpurun_out/fx2/*.
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/fx2; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "q31 or fixed or rfft or mfcc" --timeout 120 \
  --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
tail -2 $O/tests.log
for rep in 1 2; do
  for L in cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so cmsis-dsp_amd/lib/variants/lib_headfx.so; do
    v=$(basename $L .so)
    for wl in rfft_q31 mfcc_q31; do
      CMSISDSP_MI355X_LIB=$PWD/$L timeout -k 10 200 python -u bench.py --workload $wl --no-cpu-baseline > $O/${v}_${wl}_$rep.json 2> $O/${v}_${wl}_$rep.err
      python -c "import json;d=json.load(open('$O/${v}_${wl}_$rep.json'));print('$v $wl',d['value'],d['roofline'].get('avg_kernel_ms'),d['parity'].get('bit_exact'))"
    done
  done
done
