#!/bin/bash
# One GPU call: new-kernel tests first (int8 + conv), then wgrad timing and the flagship bench.
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_quantized_gpu.py -x -q > gpurun_out/pytest_quant.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_quant.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q -k "conv_fwd_dgrad_wgrad or linear" > gpurun_out/pytest_conv.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_conv.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_conv.py --iters 10 --no-miopen --ops wgrad > gpurun_out/ab_wgrad.log 2>&1 || { tail -5 gpurun_out/ab_wgrad.log; exit 3; }
tail -1 gpurun_out/ab_wgrad.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench1.log 2>&1 && tail -1 gpurun_out/bench1.log
