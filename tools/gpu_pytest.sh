#!/bin/bash
# GPU test tier only (one process), log under gpurun_out/.
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
python setup.py build_ext --inplace > gpurun_out/build.log 2>&1 || { echo build failed; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_gpu.log
exit $rc
