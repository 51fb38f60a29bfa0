#!/bin/bash
set -u
export PYTHONPATH=$PWD:${PYTHONPATH:-}
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/pytest_gpu.log | tail -8
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python tools/bench_conv.py --iters 5 > gpurun_out/bench_conv.log 2>&1 || { echo "bench_conv failed"; tail -20 gpurun_out/bench_conv.log; exit 3; }
tail -2 gpurun_out/bench_conv.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench1.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench1.log; exit 6; }
tail -1 gpurun_out/bench1.log
