set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_transformer_gpu.py tests/test_conv_family_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_e.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_e.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/diag_fork_graph.py > gpurun_out/diag_fork.log 2>&1; tail -8 gpurun_out/diag_fork.log
