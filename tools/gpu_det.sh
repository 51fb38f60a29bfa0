#!/bin/bash
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_detection_gpu.py -x -q > gpurun_out/pytest_det.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_det.log
exit $rc
