# int8 / bf16 inference throughput (Caffe-loaded ResNet-50 and Inception-v3, batch 256)
export PYTHONPATH=$PWD
for m in resnet50 inception_v3; do
  for mode in int8 bf16; do
    timeout -k 10 300 python -u tools/bench_inference.py --model $m --mode $mode > gpurun_out/inf_${m}_$mode.log 2>&1 || { tail -5 gpurun_out/inf_${m}_$mode.log; exit 1; }
    echo "$m $mode $(tail -1 gpurun_out/inf_${m}_$mode.log | grep -o '"value": [0-9.]*, "unit": "[^"]*", "n_gpus": 1, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*')"
  done
done
