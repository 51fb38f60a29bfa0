set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_conv_family_gpu.py tests/test_quantized_gpu.py tests/test_int8_graph_gpu.py tests/test_models_gpu.py tests/test_tensor_math_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_z.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_z.log
[ $rc -eq 0 ] || exit $rc
for m in inception_v3 resnet50; do
  for mode in int8 bf16; do
    timeout -k 10 300 python -u tools/bench_inference.py --model $m --mode $mode > gpurun_out/inf_${m}_${mode}.log 2>&1 || { tail -20 gpurun_out/inf_${m}_${mode}.log; exit 1; }
    echo "$m $mode $(tail -1 gpurun_out/inf_${m}_${mode}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_z.log 2>&1 || { tail -20 gpurun_out/bench_z.log; exit 1; }
echo "train $(tail -1 gpurun_out/bench_z.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"]["graph_vs_eager"])')"
