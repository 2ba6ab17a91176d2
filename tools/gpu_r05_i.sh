#!/bin/bash
# Round-5 GPU step I: RFFT-1024 p-scratch split with 16-B output stores (bin pairs per lane), A/B
# against the 8-B-store kernel, parity from the bench (out bit-exact vs the reference build).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/i1; mkdir -p $O
step() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "step rc=$rc: $*"; exit $rc; }; }
show() { python -c "import json;d=json.load(open('$1'));p=d['parity'];print('$2',d['value'],d['roofline']['frac'],d['roofline']['avg_kernel_ms'],p.get('bit_exact',p) if isinstance(p,dict) else p)"; }
lib() { [ $1 = default ] && echo cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so || echo cmsis-dsp_amd/lib/variants/lib_$1.so; }
PT="-x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
CMSISDSP_MI355X_LIB=$(lib rfst16) step 300 python -u -m pytest tests/test_gpu_rfft_fir_mat.py -k rfft $PT > $O/t_rfst16.log 2>&1
echo "rfst16 tests: $(tail -1 $O/t_rfst16.log)"
for rep in 1 2 3; do
for v in default rfst16 rfst16t4; do
  CMSISDSP_MI355X_LIB=$(lib $v) step 200 python -u bench.py --workload rfft_f32_pscratch --no-cpu-baseline > $O/rf_$v.json 2> $O/rf_$v.err
  show $O/rf_$v.json rfps_$v
done
done
echo all-ok
