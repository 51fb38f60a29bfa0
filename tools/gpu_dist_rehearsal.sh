#!/bin/bash
# Two ranks on the one GPU of the box over gloo (RCCL refuses two ranks on one device): exercises the multi-rank
# bench path (ZeRO-1 buckets, async reduce-scatter / all-gather, HIP kernels) end to end.
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out/dist
BIGDL_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 3 --warmup 2 --batch 64 > gpurun_out/dist/bench2.log 2>&1; rc=$?
tail -5 gpurun_out/dist/bench2.log
exit $rc
