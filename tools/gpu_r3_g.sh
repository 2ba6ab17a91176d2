#!/bin/bash
# Round-3 check G: MFCC q31/q15 parity and bench lines for each schedule: the default library
# (MI355X_MFCC_FX_MODE=1, two launches) and the mode-0 (three launches) build
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3g; mkdir -p $O
for L in cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so cmsis-dsp_amd/lib/variants/*.so; do
  v=$(basename $L .so)
  CMSISDSP_MI355X_LIB=$PWD/$L timeout -k 10 300 python -u -m pytest tests/test_mfcc_q31.py tests/test_mfcc_q15.py \
    -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests_$v.log 2>&1
  echo "$v: $(tail -1 $O/tests_$v.log)"
  for wl in mfcc_q31 mfcc_q15; do
    CMSISDSP_MI355X_LIB=$PWD/$L timeout -k 10 200 python -u bench.py --workload $wl --no-cpu-baseline > $O/b.json 2> $O/b.err
    python -c "import json;d=json.load(open('$O/b.json'));print('$v','$wl',d['value'],d['roofline']['avg_kernel_ms'],d['parity']['bit_exact'])"
  done
done
