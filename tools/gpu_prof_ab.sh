#!/bin/bash
# Per-step kernel table + stream overlap of the ResNet-50 training bench under rocprofv3 --kernel-trace (eager), once
# per value of one environment knob:  tools/gpu_prof_ab.sh VAR "VAL_A VAL_B"  -> gpurun_out/prof_<VAR>_<VAL>_*.txt
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
ROOT=$PWD
var=$1; vals=$2
for v in $vals; do
  tag=${var}_${v}
  (cd /tmp && export TMPDIR=/tmp && cd "$ROOT" && rm -rf gpurun_out/prof_$tag && \
    env "$var=$v" timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_$tag -o run -- python3 bench.py \
    --steps 5 --warmup 3 --graph 0 > gpurun_out/prof_bench_$tag.log 2>&1) || exit 1
  db=$(ls gpurun_out/prof_$tag/*/run_results.db gpurun_out/prof_$tag/run_results.db 2>/dev/null | head -1)
  python tools/rocpd_summary.py kernels "$db" sgd4 2 5 > gpurun_out/prof_kernels_$tag.txt || exit 1
  python tools/rocpd_streams.py "$db" sgd4 2 5 > gpurun_out/prof_streams_$tag.txt || exit 1
  rm -rf gpurun_out/prof_$tag
  echo "== $tag"; head -4 gpurun_out/prof_streams_$tag.txt
done
