#!/bin/bash
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out/infer
timeout -k 10 300 python tools/bench_inference.py --model resnet50 --mode int8 --steps 10 > gpurun_out/infer/resnet50_int8.log 2>&1 || { tail -20 gpurun_out/infer/resnet50_int8.log; exit 1; }
tail -1 gpurun_out/infer/resnet50_int8.log
timeout -k 10 300 python tools/bench_inference.py --model resnet50 --mode bf16 --steps 10 > gpurun_out/infer/resnet50_bf16.log 2>&1 || { tail -20 gpurun_out/infer/resnet50_bf16.log; exit 1; }
tail -1 gpurun_out/infer/resnet50_bf16.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/infer/trace_int8
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/infer/trace_int8 -o run -- python3 tools/bench_inference.py --model inception_v3 --mode int8 --steps 3 --warmup 1 --caffe 0 > gpurun_out/infer/prof_int8.log 2>&1 || { tail -20 gpurun_out/infer/prof_int8.log; exit 1; }
