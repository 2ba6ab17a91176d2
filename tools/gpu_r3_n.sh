#!/bin/bash
# Round-3 check N: drop-in latency (after the table-range trim), conv_f32 / fir_f32 on the
# default library and the R = 8 variant.
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3n; mkdir -p $O
timeout -k 10 120 tools/latency/dropin_latency cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so oracle/_ref/libcmsisdsp_ref.so 2000 \
  > $O/latency.json
cat $O/latency.json
for L in cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so cmsis-dsp_amd/lib/variants/*.so; do
  v=$(basename $L .so)
  for wl in conv_f32 fir_f32; do
    CMSISDSP_MI355X_LIB=$PWD/$L timeout -k 10 200 python -u bench.py --workload $wl --no-cpu-baseline > $O/${v}_$wl.json 2> $O/${v}_$wl.err
    python -c "import json;d=json.load(open('$O/${v}_$wl.json'));print('$v $wl',d['value'],d['roofline'].get('avg_kernel_ms'),d['parity'].get('bit_exact'))"
  done
done
