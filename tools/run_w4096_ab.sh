export CMSISDSP_MI355X_LIB=$PWD/cmsis-dsp_amd/lib/variants/lib_w4096.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_cfft.py -m gpu -q -x -k q31 --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/w4096_tests.log 2>&1
tail -4 gpurun_out/w4096_tests.log
timeout -k 10 200 python -u bench.py --workload cfft_q31_4096 --scaling strong --global-batch 1048576 --no-cpu-baseline --steps 10 > gpurun_out/w4096_bench.json 2>gpurun_out/w4096_bench.err || exit 1
python3 tools/show_line.py gpurun_out/w4096_bench.json variant
unset CMSISDSP_MI355X_LIB
timeout -k 10 200 python -u bench.py --workload cfft_q31_4096 --scaling strong --global-batch 1048576 --no-cpu-baseline --steps 10 > gpurun_out/w4096_base.json 2>gpurun_out/w4096_base.err || exit 1
python3 tools/show_line.py gpurun_out/w4096_base.json base
