# f32 N=4096 specialist variants (tools/build_variant.sh), run on the box.
set -e
mkdir -p gpurun_out/var4k
for lib in $1; do
  if [ $lib = base ]; then L=cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so; else L=cmsis-dsp_amd/lib/variants/lib_$lib.so; fi
  CMSISDSP_MI355X_LIB=$L timeout -k 10 200 python bench.py --workload cfft_f32_1024 --fftlen ${FFTLEN:-4096} --no-cpu-baseline --no-companion > gpurun_out/var4k/${lib}.json 2> gpurun_out/var4k/${lib}.err
done
