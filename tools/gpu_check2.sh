#!/bin/bash
# tests + smoke + 1-GPU bench + rocprofv3 kernel stats
set -u
export PYTHONPATH=$PWD:${PYTHONPATH:-}
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -rf -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 5; }
tail -3 gpurun_out/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench1.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench1.log; exit 6; }
tail -5 gpurun_out/bench1.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof1 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --graph 0 > $GRAFT_REPO_ROOT/gpurun_out/prof1.log 2>&1 || { echo "rocprof failed"; tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof1.log; exit 7; }
find $GRAFT_REPO_ROOT/gpurun_out/prof1 -name "*stats*" | head
