#!/bin/bash
# Round-5 GPU step M: forward arm_rfft_q31 / q15 N = 8192 with the split fused into the inner CFFT's last
# pass — the fixed-point RFFT GPU tests on the fused build, then A/B against the two-launch variant.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/m1; mkdir -p $O
step() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step rc=$rc: $*"; exit $rc; }; }
show() { python -c "import json;d=json.load(open('$1'));p=d['parity'];print('$2',d['value'],d['roofline']['frac'],d['roofline']['avg_kernel_ms'],p.get('bit_exact',p) if isinstance(p,dict) else p)"; }
lib() { [ $1 = default ] && echo cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so || echo cmsis-dsp_amd/lib/variants/lib_$1.so; }
PT="-x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
step 400 python -u -m pytest tests/test_rfft_fixed.py tests/test_mfcc_q31.py tests/test_mfcc_q15.py tests/test_gpu_cfft.py -m gpu $PT > $O/t_fused.log 2>&1
echo "fused tests: $(tail -1 $O/t_fused.log)"
for rep in 1 2 3; do
for v in default rfunf; do
  for w in rfft_q31 rfft_q15; do
    CMSISDSP_MI355X_LIB=$(lib $v) step 200 python -u bench.py --workload $w --no-cpu-baseline > $O/${w}_$v.json 2> $O/${w}_$v.err
    show $O/${w}_$v.json ${w}_$v
  done
done
done
echo all-ok
