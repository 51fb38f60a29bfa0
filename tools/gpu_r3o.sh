set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_quantized_gpu.py tests/test_int8_graph_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_i8.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_i8.log
[ $rc -eq 0 ] || exit $rc
for m in resnet50 inception_v3; do
  timeout -k 10 300 python -u tools/bench_inference.py --model $m --mode int8 > gpurun_out/inf_${m}_i8.log 2>&1 || { tail -20 gpurun_out/inf_${m}_i8.log; exit 1; }
  echo "$m int8 $(tail -1 gpurun_out/inf_${m}_i8.log | cut -c1-200)"
done
