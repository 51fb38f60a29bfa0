export PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest tests/test_quantized_gpu.py tests/test_int8_graph_gpu.py tests/test_kernels_gpu.py -k "halo or i8 or int8" -x -q --timeout 120 --timeout-method thread > gpurun_out/i8h_t.log 2>&1; rc=$?; tail -3 gpurun_out/i8h_t.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_inf.sh
