#!/bin/bash
# Round-3 check D: the whole -m gpu suite (zero-copy drop-in staging, FMA FIR, swizzled i8
# GEMM), the drop-in latency tool, and the headline kernel's per-launch cost: the configs[1]
# kernel timed at batch 2^14 .. 2^21 (time per launch = fixed + per-transform, fitted by
# tools/launch_fit.py).  Output: gpurun_out/r3d/*.
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3d; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/gpu_tests.log 2>&1
tail -2 $O/gpu_tests.log
timeout -k 10 120 tools/latency/dropin_latency cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so oracle/_ref/libcmsisdsp_ref.so 2000 \
  > $O/latency.json
cat $O/latency.json
for k in 14 15 16 17 18 19 20 21; do
  timeout -k 10 120 python -u bench.py --batch $((1 << k)) --steps 20 --warmup 5 --no-config3 --no-cpu-baseline \
    > $O/launch_b$k.json 2> $O/launch_b$k.err
  python -c "import json;d=json.load(open('$O/launch_b$k.json'));print($k,d['roofline']['avg_kernel_ms'],d['value'],d['parity']['bit_exact'])"
done
