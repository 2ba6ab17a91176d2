set -e
mkdir -p gpurun_out/var
for lib in base u1 skip; do
  if [ $lib = base ]; then L=cmsis-dsp_amd/lib/libcmsisdsp_mi355x.so; else L=cmsis-dsp_amd/lib/variants/lib_$lib.so; fi
  CMSISDSP_MI355X_LIB=$L timeout -k 10 200 python bench.py --workload mfcc_f32 --no-cpu-baseline > gpurun_out/var/mfcc_$lib.json 2> gpurun_out/var/mfcc_$lib.err
done
