set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/firp
timeout -k 10 120 tools/probes/valu_rate > gpurun_out/firp/valu_rate.txt 2>&1 || exit $?
cat gpurun_out/firp/valu_rate.txt
for v in base fr12 fr16; do
  if [ $v = base ]; then L=cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so; else L=cmsis-dsp_amd/lib/variants/lib_$v.so; fi
  CMSISDSP_MI355X_LIB=$PWD/$L timeout -k 10 120 python -u bench.py --workload fir_f32 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/firp/fir_$v.json 2> gpurun_out/firp/fir_$v.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/firp/fir_$v.json'));print('$v',d['value'],d['roofline']['avg_kernel_ms'],d['parity']['bit_exact'])"
done
