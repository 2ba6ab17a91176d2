set -e
# Sweep fixed-point mat_mult variants (tools/build_variant.sh <name> ...).
mkdir -p gpurun_out/var
for lib in base $VARIANTS; do
  if [ $lib = base ]; then L=cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so; else L=cmsis-dsp_amd/lib/variants/lib_$lib.so; fi
  for wl in mat_mult_q15 mat_mult_q31; do
    CMSISDSP_MI355X_LIB=$L timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline > gpurun_out/var/${lib}_$wl.json 2> gpurun_out/var/${lib}_$wl.err
  done
done
