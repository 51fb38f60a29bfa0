#!/bin/bash
# Kernel-trace profiles of bench.py with an env switch on and off: tools/gpu_ab_prof.sh ENVVAR
set -o pipefail
export PYTHONPATH=$PWD
VAR=${1:-BIGDL_DGRAD_BN}
mkdir -p gpurun_out/ab
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in 1 0; do
  rm -rf gpurun_out/ab/t$v
  export $VAR=$v
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/ab/t$v -o run -- python3 bench.py --steps 5 --warmup 3 --graph 0 > gpurun_out/ab/bench$v.log 2>&1 || { echo "trace $v failed"; exit 1; }
  python3 tools/rocpd_summary.py kernels $(find gpurun_out/ab/t$v -name '*.db' | head -1) > gpurun_out/ab/k$v.txt 2>&1
  head -14 gpurun_out/ab/k$v.txt
  find gpurun_out/ab/t$v -name '*.db' -delete
done
