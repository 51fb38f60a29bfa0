#!/bin/bash
set -u
export PYTHONPATH=$PWD:${PYTHONPATH:-}
mkdir -p gpurun_out
timeout -k 10 400 python tools/bench_conv.py --iters 5 > gpurun_out/bench_conv.log 2>&1 || { echo "bench_conv failed $?"; tail -20 gpurun_out/bench_conv.log; exit 3; }
cat gpurun_out/bench_conv.log
timeout -k 10 300 python tools/torch_resnet50_ref.py > gpurun_out/torchref.log 2>&1 || { echo "torchref failed"; tail -20 gpurun_out/torchref.log; exit 4; }
cat gpurun_out/torchref.log
