set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "lrn or dropout or embedding or resize or bf16_trunc" > gpurun_out/pytest_misc.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_misc.log
exit $rc
