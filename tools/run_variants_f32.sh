#!/bin/bash
# cfft_f32 at one fftLen (FFTLEN, default 4096; bench.py --fftlen: the same 8 GiB per launch)
# on each library variant (tools/build_variant.sh) and the default library.
# Output: gpurun_out/var_f32_$FFTLEN/<variant>.json
set -o pipefail
export TMPDIR=/tmp
N=${FFTLEN:-4096}
O=gpurun_out/var_f32_$N; mkdir -p $O
for L in cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so cmsis-dsp_amd/lib/variants/*.so; do
  v=$(basename $L .so)
  CMSISDSP_MI355X_LIB=$PWD/$L timeout -k 10 120 python -u bench.py --fftlen $N --steps ${STEPS:-10} --warmup 3 \
    --no-config3 --no-cpu-baseline > $O/$v.json 2> $O/$v.err || exit $?
  python -c "import json;d=json.load(open('$O/$v.json'));print('$v',d['value'],d['roofline']['frac'],d['roofline']['avg_kernel_ms'],d['parity'].get('bit_exact'))"
done
