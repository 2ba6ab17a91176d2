set -e
mkdir -p gpurun_out/var
for lib in base tw0 tw0w3; do
  for wl in cfft_q31_4096 cfft_q15_4096; do
    if [ $lib = base ]; then L=cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so; else L=cmsis-dsp_amd/lib/variants/lib_$lib.so; fi
    CMSISDSP_MI355X_LIB=$L timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline > gpurun_out/var/${lib}_$wl.json 2> gpurun_out/var/${lib}_$wl.err
  done
done
