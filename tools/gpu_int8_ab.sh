# int8 inference A/B of one knob: tests, per-layer int8 roofline and bench_inference for each value
export PYTHONPATH=$PWD
var=${1:-BIGDL_I8_EPI}; vals=${2:-"1 0"}
timeout -k 10 400 python -u -m pytest tests/test_quantized_gpu.py tests/test_int8_graph_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/i8ab_test.log 2>&1; rc=$?; tail -2 gpurun_out/i8ab_test.log; [ $rc -eq 0 ] || exit $rc
for v in $vals; do
  env $var=$v timeout -k 10 300 python -u tools/int8_roofline.py > gpurun_out/i8roof_$v.log 2>&1 || { tail -5 gpurun_out/i8roof_$v.log; exit 1; }
  echo "$var=$v $(tail -1 gpurun_out/i8roof_$v.log)"
  for m in resnet50 inception_v3; do
    env $var=$v timeout -k 10 300 python -u tools/bench_inference.py --model $m --mode int8 > gpurun_out/i8ab_${m}_$v.log 2>&1 || { tail -5 gpurun_out/i8ab_${m}_$v.log; exit 1; }
    echo "$var=$v $m $(tail -1 gpurun_out/i8ab_${m}_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done
