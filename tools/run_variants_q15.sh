set -e
mkdir -p gpurun_out/var
for lib in base w4; do
  if [ $lib = base ]; then L=cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so; else L=cmsis-dsp_amd/lib/variants/lib_$lib.so; fi
  CMSISDSP_MI355X_LIB=$L timeout -k 10 200 python bench.py --workload cfft_q15_4096 --no-cpu-baseline > gpurun_out/var/q15_$lib.json 2> gpurun_out/var/q15_$lib.err
done
timeout -k 10 200 python bench.py --workload cfft_q31_4096 --no-cpu-baseline > gpurun_out/var/q31_base.json 2> gpurun_out/var/q31_base.err
