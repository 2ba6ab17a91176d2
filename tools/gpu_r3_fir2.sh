#!/bin/bash
# FIR f32 look-ahead coefficient schedule: FIR / conv / decimate GPU parity, then the fir_f32 and
# conv_f32 bench lines of the new library and of the previous kernel (lib_headfir variant),
# alternated twice.  Output: gpurun_out/fir2/*.
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/fir2; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "fir or conv or correlate or decim or interp" --timeout 120 \
  --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
tail -2 $O/tests.log
for rep in 1 2; do
  for L in cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so cmsis-dsp_amd/lib/variants/lib_headfir.so; do
    v=$(basename $L .so)
    for wl in fir_f32 conv_f32; do
      CMSISDSP_MI355X_LIB=$PWD/$L timeout -k 10 200 python -u bench.py --workload $wl --no-cpu-baseline > $O/${v}_${wl}_$rep.json 2> $O/${v}_${wl}_$rep.err
      python -c "import json;d=json.load(open('$O/${v}_${wl}_$rep.json'));print('$v $wl',d['value'],d['roofline'].get('avg_kernel_ms'),d['parity'].get('bit_exact'))"
    done
  done
done
