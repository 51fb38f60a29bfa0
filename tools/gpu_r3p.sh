set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_tensor_math_gpu.py tests/test_models_gpu.py tests/test_graph_fusion_gpu.py tests/test_quantized_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_p.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_p.log
[ $rc -eq 0 ] || exit $rc
for m in resnet50 inception_v3; do
  for mode in bf16 int8; do
    timeout -k 10 300 python -u tools/bench_inference.py --model $m --mode $mode > gpurun_out/inf_${m}_${mode}.log 2>&1 || { tail -20 gpurun_out/inf_${m}_${mode}.log; exit 1; }
    echo "$m $mode $(tail -1 gpurun_out/inf_${m}_${mode}.log | cut -c1-200)"
  done
done
