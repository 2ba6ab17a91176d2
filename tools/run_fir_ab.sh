set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/fir1
timeout -k 10 300 python -u -m pytest tests -m gpu -q -k "fir" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/fir1/tests.log 2>&1; rc=$?
tail -3 gpurun_out/fir1/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2; do timeout -k 10 200 python -u bench.py --workload fir_f32 --no-cpu-baseline > gpurun_out/fir1/bench$i.json 2>gpurun_out/fir1/bench$i.err || exit $?; python -c "import json;d=json.load(open('gpurun_out/fir1/bench$i.json'));print(d['value'],d['ms_per_step'],d['roofline'])"; done
exit $rc
