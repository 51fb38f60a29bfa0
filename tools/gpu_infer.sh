#!/bin/bash
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out/infer
timeout -k 10 300 python -u -m pytest tests/test_quantized_gpu.py tests/test_models_gpu.py -q -x --timeout 200 --timeout-method thread -k "quant or inception_v3 or ir_dnn" > gpurun_out/infer/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/infer/pytest.log
[ $rc -eq 0 ] || exit $rc
for cfg in "inception_v3 int8" "inception_v3 bf16" "resnet50 int8" "resnet50 bf16"; do
  set -- $cfg
  timeout -k 10 300 python tools/bench_inference.py --model $1 --mode $2 --steps 10 > gpurun_out/infer/$1_$2.log 2>&1 || { tail -20 gpurun_out/infer/$1_$2.log; exit 1; }
  tail -1 gpurun_out/infer/$1_$2.log
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/infer/trace_int8
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/infer/trace_int8 -o run -- python3 tools/bench_inference.py --model inception_v3 --mode int8 --steps 3 --warmup 1 --caffe 0 > gpurun_out/infer/prof_int8.log 2>&1 || { tail -20 gpurun_out/infer/prof_int8.log; exit 1; }
