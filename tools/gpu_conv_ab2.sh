#!/bin/bash
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q -k "conv" > gpurun_out/pytest_conv.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_conv.log
[ $rc -eq 0 ] || exit $rc
for impl in 0 1 2; do
  BIGDL_CONV_IMPL=$impl timeout -k 10 300 python tools/bench_conv.py --iters 10 --no-miopen --ops fwd,dgrad > gpurun_out/ab_impl$impl.log 2>&1 || { echo "bench impl $impl failed"; tail -5 gpurun_out/ab_impl$impl.log; exit 3; }
  echo "impl $impl: $(tail -1 gpurun_out/ab_impl$impl.log)"
done
BIGDL_CONV_IMPL=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_impl1.log 2>&1 && tail -1 gpurun_out/bench_impl1.log
