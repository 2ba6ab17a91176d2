#!/bin/bash
# Library variant sweep on one MI355X: bench.py --workload $WL (default fir_f32) against each library
# variant in cmsis-dsp_amd/lib/variants (tools/build_variant.sh) and the default library.
# Output: gpurun_out/var_${WL:-fir_f32}/*.json
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/var_${WL:-fir_f32}
for L in cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so cmsis-dsp_amd/lib/variants/*.so; do
  v=$(basename $L .so)
  CMSISDSP_MI355X_LIB=$PWD/$L timeout -k 10 120 python -u bench.py --workload ${WL:-fir_f32} --steps ${STEPS:-10} --warmup 3 --no-config3 ${ARGS} \
    --no-cpu-baseline > gpurun_out/var_${WL:-fir_f32}/$v.json 2> gpurun_out/var_${WL:-fir_f32}/$v.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/var_${WL:-fir_f32}/$v.json'));print('$v',d['value'],d['roofline']['avg_kernel_ms'],d['parity'].get('bit_exact'))"
done
