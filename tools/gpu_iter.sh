export PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "s1_stream or g4_kernel or p8_kernel or fwd_dgrad_wgrad" > gpurun_out/t5.log 2>&1; rc=$?; tail -5 gpurun_out/t5.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/conv_variants.py --layers 1,3,4,5,7,9 --variants "s1:s1=1;old:s1=0" > gpurun_out/v5.log 2>&1; rc=$?; cat gpurun_out/v5.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/b5.log 2>&1; rc=$?; tail -1 gpurun_out/b5.log | cut -c1-400; exit $rc
