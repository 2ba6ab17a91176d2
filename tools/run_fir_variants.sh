#!/bin/bash
# fir_f32 (bit-exact) and fir_f32_fma bench lines on the default library and every variant in
# cmsis-dsp_amd/lib/variants (tools/build_variant.sh).  Output: gpurun_out/fir_var/*.
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/fir_var; mkdir -p $O
for L in cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so cmsis-dsp_amd/lib/variants/*.so; do
  v=$(basename $L .so)
  for wl in fir_f32 fir_f32_fma; do
    CMSISDSP_MI355X_LIB=$PWD/$L timeout -k 10 120 python -u bench.py --workload $wl --no-cpu-baseline \
      > $O/${v}_$wl.json 2> $O/${v}_$wl.err
    python -c "import json;d=json.load(open('$O/${v}_$wl.json'));print('$v $wl',d['value'],d['roofline']['avg_kernel_ms'],d['parity'].get('bit_exact'),d['parity'].get('within_bound'))"
  done
done
