#!/bin/bash
# MFCC f32 Mel stage regrouped per (filter, frame): MFCC GPU parity, then mfcc_f32 bench lines of
# the new library and of the previous kernel (lib_headmfcc), alternated.  Output: gpurun_out/mfcc2/*.
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/mfcc2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "mfcc" --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/tests.log 2>&1
tail -2 $O/tests.log
for rep in 1 2; do
  for L in cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so cmsis-dsp_amd/lib/variants/lib_headmfcc.so; do
    v=$(basename $L .so)
    CMSISDSP_MI355X_LIB=$PWD/$L timeout -k 10 200 python -u bench.py --workload mfcc_f32 --no-cpu-baseline > $O/${v}_$rep.json 2> $O/${v}_$rep.err
    python -c "import json;d=json.load(open('$O/${v}_$rep.json'));print('$v',d['value'],d['roofline'].get('avg_kernel_ms'),d['parity'].get('bit_exact'))"
  done
done
