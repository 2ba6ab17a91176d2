#!/bin/bash
# Round-5 GPU step V: the fused radix-16 forward RFFT q31 at fftLenReal 2048 with its registers capped
# at three waves per SIMD (MI355X_RFFT_SPLIT_WAVES1024=3, 4 VGPRs spilled) against the default's two;
# then the current library's RFFT GPU tests (N = 256 inverse register cap) and its inverse timing.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/v1; mkdir -p $O
step() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step rc=$rc: $*"; exit $rc; }; }
show() { python -c "import json;d=json.load(open('$1'));p=d['parity'];print('$2',d['value'],d['roofline']['frac'],d['roofline']['avg_kernel_ms'],p.get('bit_exact',p) if isinstance(p,dict) else p)"; }
lib() { [ $1 = default ] && echo cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so || echo cmsis-dsp_amd/lib/variants/lib_$1.so; }
PT="-x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
for v in default rs3; do
  CMSISDSP_MI355X_LIB=$(lib $v) step 400 python -u -m pytest tests/test_rfft_fixed.py -m gpu $PT > $O/t_$v.log 2>&1
  echo "$v tests: $(tail -1 $O/t_$v.log)"
done
for rep in 1 2 3; do
for v in default rs3; do
  CMSISDSP_MI355X_LIB=$(lib $v) step 200 python -u bench.py --workload rfft_q31 --fftlen 2048 --no-cpu-baseline > $O/q31_2048_${v}_$rep.json 2> $O/q31_2048_${v}_$rep.err
  show $O/q31_2048_${v}_$rep.json rfft_q31_2048_$v
done
done
step 300 python -u tools/rfft_inv_ab.py 512 1024 2048 4096 8192 > $O/inv_default.txt 2>&1
grep "^q" $O/inv_default.txt
echo all-ok
