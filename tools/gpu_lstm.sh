set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_recurrent_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_lstm.log 2>&1; rc=$?
tail -25 gpurun_out/pytest_lstm.log
exit $rc
