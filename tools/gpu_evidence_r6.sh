#!/bin/bash
# Round-6 evidence runs on one GPU box: the LSTM LM (config 5) at batch 128 / 256 and the Caffe-loaded inference
# benches (config 4 + ResNet-50), one JSON line each -> gpurun_out/r6_*.json(l)
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_lstm.py --steps 10 --warmup 3 --batch 128 > gpurun_out/r6_lstm_lm_b128.log 2>&1 || exit 1
tail -1 gpurun_out/r6_lstm_lm_b128.log > gpurun_out/r6_lstm_lm_b128.json
timeout -k 10 300 python tools/bench_lstm.py --steps 10 --warmup 3 --batch 256 > gpurun_out/r6_lstm_lm_b256.log 2>&1 || exit 1
tail -1 gpurun_out/r6_lstm_lm_b256.log > gpurun_out/r6_lstm_lm_b256.json
rm -f gpurun_out/r6_inference_benches.jsonl
for m in inception_v3 resnet50; do
  for mode in int8 bf16; do
    timeout -k 10 400 python tools/bench_inference.py --model $m --mode $mode > gpurun_out/r6_inf_${m}_${mode}.log 2>&1 || exit 1
    tail -1 gpurun_out/r6_inf_${m}_${mode}.log >> gpurun_out/r6_inference_benches.jsonl
  done
done
cut -c1-220 gpurun_out/r6_lstm_lm_b128.json gpurun_out/r6_lstm_lm_b256.json gpurun_out/r6_inference_benches.jsonl
