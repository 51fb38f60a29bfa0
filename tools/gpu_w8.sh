set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "w8 or conv" > gpurun_out/pytest_w8.log 2>&1 || { tail -30 gpurun_out/pytest_w8.log; exit 1; }
tail -3 gpurun_out/pytest_w8.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_w8.log 2>&1 || { tail -20 gpurun_out/bench_w8.log; exit 1; }
tail -1 gpurun_out/bench_w8.log
BIGDL_CONV_W8=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_now8.log 2>&1 && tail -1 gpurun_out/bench_now8.log
timeout -k 10 300 python tools/bench_conv.py --no-miopen --ops fwd,dgrad > gpurun_out/bench_conv_w8.log 2>&1 && tail -1 gpurun_out/bench_conv_w8.log
BIGDL_CONV_W8=0 timeout -k 10 300 python tools/bench_conv.py --no-miopen --ops fwd,dgrad > gpurun_out/bench_conv_now8.log 2>&1 && tail -1 gpurun_out/bench_conv_now8.log
