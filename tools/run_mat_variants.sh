#!/bin/bash
# mat_mult_q15 / q31 bench lines on the default library and every variant in
# cmsis-dsp_amd/lib/variants.  Output: gpurun_out/mat_var/*.
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/mat_var; mkdir -p $O
for L in cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so cmsis-dsp_amd/lib/variants/*.so; do
  v=$(basename $L .so)
  for wl in mat_mult_q15 mat_mult_q31; do
    CMSISDSP_MI355X_LIB=$PWD/$L timeout -k 10 200 python -u bench.py --workload $wl --no-cpu-baseline > $O/${v}_$wl.json 2> $O/${v}_$wl.err
    python -c "import json;d=json.load(open('$O/${v}_$wl.json'));print('$v $wl',d['value'],d['roofline'].get('avg_kernel_ms'),d['parity'].get('bit_exact'))"
  done
done
