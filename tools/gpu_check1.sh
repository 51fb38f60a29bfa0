#!/bin/bash
# round-1 first hardware check: kernel numerics, per-layer conv timing, vendor calibration point
set -u
export PYTHONPATH=$PWD:${PYTHONPATH:-}
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 500 python -m pytest tests/test_kernels_gpu.py -q -rf > gpurun_out/kt.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -40 gpurun_out/kt.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/bench_conv.py --iters 5 > gpurun_out/bench_conv.log 2>&1 || { echo "bench_conv failed $?"; tail -20 gpurun_out/bench_conv.log; exit 3; }
tail -30 gpurun_out/bench_conv.log
timeout -k 10 240 python tools/torch_resnet50_ref.py > gpurun_out/torchref.log 2>&1 || { echo "torchref failed"; tail -20 gpurun_out/torchref.log; exit 4; }
cat gpurun_out/torchref.log
