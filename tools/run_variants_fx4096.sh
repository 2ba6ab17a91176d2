#!/bin/bash
# q31 / q15 N=4096 strong-scaling (2^20 transforms) on each library variant
# (cmsis-dsp_amd/lib/variants, tools/build_variant.sh) and the default library.
# Output: gpurun_out/var_fx4096/<variant>_<q31|q15>.json
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/var_fx4096; mkdir -p $O
for L in cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so cmsis-dsp_amd/lib/variants/*.so; do
  v=$(basename $L .so)
  for ty in q31 q15; do
    CMSISDSP_MI355X_LIB=$PWD/$L timeout -k 10 120 python -u bench.py --workload cfft_${ty}_4096 --scaling strong \
      --global-batch 1048576 --steps ${STEPS:-8} --warmup 3 --no-config3 --no-cpu-baseline > $O/${v}_$ty.json 2> $O/${v}_$ty.err || exit $?
    python -c "import json;d=json.load(open('$O/${v}_$ty.json'));print('$v $ty',d['value'],d['roofline']['frac'],d['roofline']['avg_kernel_ms'],d['parity'].get('bit_exact'))"
  done
done
