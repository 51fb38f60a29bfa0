#!/bin/bash
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q -k "conv" > gpurun_out/pytest_conv.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_conv.log
[ $rc -eq 0 ] || exit $rc
BIGDL_CONV_IMPL=0 timeout -k 10 300 python tools/bench_conv.py --iters 10 --no-miopen --ops wgrad > gpurun_out/ab_wgrad0.log 2>&1 || { tail -5 gpurun_out/ab_wgrad0.log; exit 3; }
tail -1 gpurun_out/ab_wgrad0.log
BIGDL_CONV_IMPL=1 timeout -k 10 300 python tools/bench_conv.py --iters 10 --no-miopen --ops wgrad > gpurun_out/ab_wgrad1.log 2>&1 || { tail -5 gpurun_out/ab_wgrad1.log; exit 3; }
tail -1 gpurun_out/ab_wgrad1.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench1.log 2>&1 && tail -1 gpurun_out/bench1.log
