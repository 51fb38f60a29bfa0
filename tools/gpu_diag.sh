#!/bin/bash
set -u
export PYTHONPATH=$PWD:${PYTHONPATH:-}
mkdir -p gpurun_out
timeout -k 10 300 python tools/diag_layers.py --fuse 1 > gpurun_out/diag_fused.log 2>&1 || { tail -20 gpurun_out/diag_fused.log; exit 3; }
timeout -k 10 300 python tools/diag_layers.py --fuse 0 > gpurun_out/diag_unfused.log 2>&1 || { tail -20 gpurun_out/diag_unfused.log; exit 4; }
echo done
