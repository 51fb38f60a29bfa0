#!/bin/bash
# Kernel tests matching $1, then one rocprofv3 kernel-trace of bench.py (eager) summarised to gpurun_out/q/kernels.txt
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out/q
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "${1:-transpose}" --timeout 120 --timeout-method thread > gpurun_out/q/pt.log 2>&1; rc=$?
tail -2 gpurun_out/q/pt.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/q/t
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/q/t -o run -- python3 bench.py --steps 5 --warmup 3 --graph 0 > gpurun_out/q/bench.log 2>&1 || { echo "trace failed"; exit 1; }
python3 tools/rocpd_summary.py kernels $(find gpurun_out/q/t -name '*.db' | head -1) > gpurun_out/q/kernels.txt 2>&1
find gpurun_out/q/t -name '*.db' -delete
head -16 gpurun_out/q/kernels.txt | cut -c1-110
