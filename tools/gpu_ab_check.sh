#!/bin/bash
# Targeted GPU check + A/B bench of an env switch: tools/gpu_ab_check.sh ENVVAR "pytest -k expr" ON OFF
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
VAR=${1:-BIGDL_DGRAD_BN}
K=${2:-"bottleneck or resnet_gpu or dgrad_epilogue or bn"}
ON=${3:-1}
OFF=${4:-0}
timeout -k 10 400 python -u -m pytest tests/test_models_gpu.py tests/test_kernels_gpu.py -x -q -k "$K" --timeout 200 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_ab.log
[ $rc -eq 0 ] || exit $rc
env $VAR=$ON timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_on.log 2>&1 || exit 1
tail -1 gpurun_out/bench_on.log
env $VAR=$OFF timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_off.log 2>&1 || exit 1
tail -1 gpurun_out/bench_off.log
