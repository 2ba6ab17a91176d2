set -o pipefail
mkdir -p gpurun_out/sp
timeout -k 10 300 python -u -m pytest tests/test_rfft_fixed.py tests/test_mfcc_q31.py tests/test_pythonwrapper_compat.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/sp/tests.log 2>&1
rc=$?; tail -3 gpurun_out/sp/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for w in mfcc_q31 rfft_q31 rfft_q15; do
  timeout -k 10 200 python -u bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/sp/$w.json 2> gpurun_out/sp/$w.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/sp/$w.json'));print('$w',d['value'],d['roofline']['frac'],d['parity'])"
done
