set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_conv_family_gpu.py tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_pair.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_pair.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_pair.log 2>&1 || { tail -20 gpurun_out/bench_pair.log; exit 1; }
tail -1 gpurun_out/bench_pair.log
bash tools/gpu_run.sh prof
