#!/bin/bash
# Round-5 GPU step T: the one-launch MFCC q15 / q31 schedule (MI355X_MFCC_FX_MODE=2) at 3 / 4 waves
# per SIMD (MI355X_MQF_WG) and 8 / 16 groups per workgroup (MI355X_FXR_T), against the two-launch
# default: the MFCC fixed-point GPU tests on each variant, then two alternating bench lines.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/t1; mkdir -p $O
step() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step rc=$rc: $*"; exit $rc; }; }
show() { python -c "import json;d=json.load(open('$1'));p=d['parity'];r=d['roofline'];print('$2',d['value'],r['frac'],r['avg_kernel_ms'],r.get('traffic'),p.get('bit_exact',p) if isinstance(p,dict) else p)"; }
lib() { [ $1 = default ] && echo cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so || echo cmsis-dsp_amd/lib/variants/lib_$1.so; }
PT="-x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
VS="m2wg3 m2wg4 m2wg3t16 m2wg4t16"
for v in $VS; do
  CMSISDSP_MI355X_LIB=$(lib $v) step 300 python -u -m pytest tests/test_mfcc_q31.py tests/test_mfcc_q15.py -m gpu $PT > $O/t_$v.log 2>&1
  echo "$v tests: $(tail -1 $O/t_$v.log)"
done
for rep in 1 2; do
for v in default $VS; do
  for w in mfcc_q15 mfcc_q31; do
    CMSISDSP_MI355X_LIB=$(lib $v) step 200 python -u bench.py --workload $w --no-cpu-baseline > $O/${w}_${v}_$rep.json 2> $O/${w}_${v}_$rep.err
    show $O/${w}_${v}_$rep.json ${w}_$v
  done
done
done
echo all-ok
