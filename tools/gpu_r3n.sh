set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_tensor_math_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_tm.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_tm.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_r3m.sh
