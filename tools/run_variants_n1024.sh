set -e
# Sweep cfft_f32 N=1024 work-mapping variants (tools/build_variant.sh n<name> ...).
mkdir -p gpurun_out/var
for lib in base $VARIANTS; do
  if [ $lib = base ]; then L=cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so; else L=cmsis-dsp_amd/lib/variants/lib_$lib.so; fi
  CMSISDSP_MI355X_LIB=$L timeout -k 10 200 python bench.py --workload cfft_f32_1024 --no-cpu-baseline > gpurun_out/var/${lib}_n1024.json 2> gpurun_out/var/${lib}_n1024.err
done
