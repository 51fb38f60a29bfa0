#!/bin/bash
# Halo weight gradient in atomic split mode (BIGDL_WGRAD_HALO_ATOMIC=1): its numerics tests, then an interleaved
# bench A/B against the workspace + halo_reduce_kernel path.
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
BIGDL_WGRAD_HALO_ATOMIC=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py -k "wgrad" > gpurun_out/halo_atomic_tests.log 2>&1 || { tail -30 gpurun_out/halo_atomic_tests.log; exit 1; }
tail -2 gpurun_out/halo_atomic_tests.log
bash tools/gpu_ab_knobs.sh "BIGDL_WGRAD_HALO_ATOMIC=0" "BIGDL_WGRAD_HALO_ATOMIC=1"
