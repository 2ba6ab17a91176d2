#!/bin/bash
# Round-5 GPU step K: RFFT-1024 split with bin k from the stage-2 registers (only bin 512 - k from
# LDS): rfft bit-exact tests, then A/B against the default, same box.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/k1; mkdir -p $O
step() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step rc=$rc: $*"; exit $rc; }; }
show() { python -c "import json;d=json.load(open('$1'));p=d['parity'];print('$2',d['value'],d['roofline']['frac'],d['roofline']['avg_kernel_ms'],p.get('bit_exact',p) if isinstance(p,dict) else p)"; }
lib() { [ $1 = default ] && echo cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so || echo cmsis-dsp_amd/lib/variants/lib_$1.so; }
PT="-x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
CMSISDSP_MI355X_LIB=$(lib rfreg) step 300 python -u -m pytest tests/test_gpu_rfft_fir_mat.py -k rfft $PT > $O/t_rfreg.log 2>&1
echo "rfreg tests: $(tail -1 $O/t_rfreg.log)"
for rep in 1 2 3; do
for v in default rfreg; do
  for w in rfft_f32_pscratch rfft_f32; do
    CMSISDSP_MI355X_LIB=$(lib $v) step 200 python -u bench.py --workload $w --no-cpu-baseline > $O/${w}_$v.json 2> $O/${w}_$v.err
    show $O/${w}_$v.json ${w}_$v
  done
done
done
echo all-ok
