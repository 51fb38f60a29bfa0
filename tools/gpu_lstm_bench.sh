#!/bin/bash
# LSTM tests + LM bench (graph) + kernel-time profile of the eager step.
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out/lstm
timeout -k 10 300 python -u -m pytest tests/test_recurrent_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "lstm or softmax or LSTM" > gpurun_out/lstm/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/lstm/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/bench_lstm.py --steps 5 --warmup 2 > gpurun_out/lstm/bench.log 2>&1; rc=$?
tail -3 gpurun_out/lstm/bench.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/lstm/trace
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/lstm/trace -o run -- python3 tools/bench_lstm.py --steps 2 --warmup 1 --graph 0 > gpurun_out/lstm/prof.log 2>&1 || { echo "trace failed"; tail -20 gpurun_out/lstm/prof.log; exit 1; }
