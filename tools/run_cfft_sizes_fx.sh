#!/bin/bash
# q31 / q15 CFFT throughput at every length 16..4096 (same bytes per launch as configs[3]).
# Output: gpurun_out/sizes_fx/<type>_<N>.json and a summary line per run.
set -o pipefail
mkdir -p gpurun_out/sizes_fx
for ty in q31 q15; do
  for n in ${SIZES:-16 32 64 128 256 512 1024 2048 4096}; do
    timeout -k 10 120 python -u bench.py --workload cfft_${ty}_4096 --fftlen $n --steps 10 --warmup 3 --no-cpu-baseline \
      --no-config3 > gpurun_out/sizes_fx/${ty}_$n.json 2> gpurun_out/sizes_fx/${ty}_$n.err || exit $?
    python -c "import json;d=json.load(open('gpurun_out/sizes_fx/${ty}_$n.json'));print('$ty $n',d['value'],d['roofline']['frac'],d['parity'].get('bit_exact'))"
  done
done
