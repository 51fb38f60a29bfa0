#!/bin/bash
# LSTM LM (config 5, batch 128) per-step kernel table under rocprofv3 --kernel-trace (eager): last 3 of 5 steps
set -o pipefail
export PYTHONPATH=$PWD
ROOT=$PWD
mkdir -p gpurun_out
(cd /tmp && export TMPDIR=/tmp && cd "$ROOT" && rm -rf gpurun_out/lstmprof && \
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/lstmprof -o run -- python3 tools/bench_lstm.py --steps 5 \
  --warmup 2 --batch 128 --graph 0 > gpurun_out/lstm_prof.log 2>&1) || { tail -20 gpurun_out/lstm_prof.log; exit 1; }
db=$(ls gpurun_out/lstmprof/*/run_results.db gpurun_out/lstmprof/run_results.db 2>/dev/null | head -1)
python tools/rocpd_summary.py kernels "$db" sgd4 4 3 > gpurun_out/lstm_kernels_per_step.txt || exit 1
python tools/rocpd_streams.py "$db" sgd4 4 3 > gpurun_out/lstm_streams.txt || exit 1
rm -rf gpurun_out/lstmprof
head -30 gpurun_out/lstm_kernels_per_step.txt | cut -c1-150
head -4 gpurun_out/lstm_streams.txt
