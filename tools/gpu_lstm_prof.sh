#!/bin/bash
# LSTM LM (config 5) bench + rocprofv3 kernel table (eager, so every kernel is attributed).
set -o pipefail
export PYTHONPATH=$PWD
ROOT=$PWD
mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_lstm.py --steps 10 --warmup 3 --batch 64 > gpurun_out/lstm_b64.log 2>&1 || { tail -20 gpurun_out/lstm_b64.log; exit 1; }
tail -1 gpurun_out/lstm_b64.log
timeout -k 10 300 python tools/bench_lstm.py --steps 10 --warmup 3 --batch 128 > gpurun_out/lstm_b128.log 2>&1 || { tail -20 gpurun_out/lstm_b128.log; exit 1; }
tail -1 gpurun_out/lstm_b128.log
(cd /tmp && export TMPDIR=/tmp && cd "$ROOT" && rm -rf gpurun_out/lstmprof && \
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/lstmprof -o run -- python3 tools/bench_lstm.py --steps 2 --warmup 1 --batch 64 --graph 0 \
  > gpurun_out/lstm_prof.log 2>&1) || { tail -20 gpurun_out/lstm_prof.log; exit 1; }
tail -1 gpurun_out/lstm_prof.log
