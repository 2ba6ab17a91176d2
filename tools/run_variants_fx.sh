set -e
# Sweep cfft_q31/q15 N=4096 variants (tools/build_variant.sh <name> ...).
mkdir -p gpurun_out/var
for lib in base $VARIANTS; do
  if [ $lib = base ]; then L=cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so; else L=cmsis-dsp_amd/lib/variants/lib_$lib.so; fi
  for wl in cfft_q31_4096 cfft_q15_4096; do
    CMSISDSP_MI355X_LIB=$L timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline > gpurun_out/var/${lib}_$wl.json 2> gpurun_out/var/${lib}_$wl.err
  done
done
