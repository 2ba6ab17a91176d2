mkdir -p gpurun_out/ab1
for rep in 1 2; do
  for v in default q7l q7pp1; do
    if [ $v = default ]; then
      timeout -k 10 120 python bench.py --workload mat_mult_q7 --steps 10 --warmup 3 > gpurun_out/ab1/$v.$rep.json 2>/dev/null || exit 1
    else
      CMSISDSP_MI355X_LIB=cmsis-dsp_amd/lib/variants/lib_$v.so timeout -k 10 120 python bench.py --workload mat_mult_q7 --steps 10 --warmup 3 > gpurun_out/ab1/$v.$rep.json 2>/dev/null || exit 1
    fi
  done
done
