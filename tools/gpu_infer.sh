#!/bin/bash
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out/infer
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py -q -x --timeout 200 --timeout-method thread -k "inception_v3" > gpurun_out/infer/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/infer/pytest.log
[ $rc -eq 0 ] || exit $rc
for cfg in "inception_v3 int8" "inception_v3 bf16" "resnet50 int8" "resnet50 bf16"; do
  set -- $cfg
  timeout -k 10 300 python tools/bench_inference.py --model $1 --mode $2 --steps 10 > gpurun_out/infer/$1_$2.log 2>&1 || { tail -20 gpurun_out/infer/$1_$2.log; exit 1; }
  tail -1 gpurun_out/infer/$1_$2.log
done
