#!/bin/bash
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/prof/trace
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace -o run -- python3 bench.py --steps 5 --warmup 3 --graph 0 > gpurun_out/prof/bench.log 2>&1 || { echo "trace run failed"; tail -20 gpurun_out/prof/bench.log; exit 1; }
tail -1 gpurun_out/prof/bench.log
