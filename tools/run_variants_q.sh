# q31/q15 N=4096 specialist variants: tools/build_variant.sh builds them, this runs them on the box.
# Usage (on the GPU box): bash tools/run_variants_q.sh "base w4 tw0 ..."
set -e
mkdir -p gpurun_out/var
for lib in $1; do
  for wl in cfft_q31_4096 cfft_q15_4096; do
    if [ $lib = base ]; then L=cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so; else L=cmsis-dsp_amd/lib/variants/lib_$lib.so; fi
    CMSISDSP_MI355X_LIB=$L timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline --no-companion > gpurun_out/var/${lib}_$wl.json 2> gpurun_out/var/${lib}_$wl.err
  done
done
