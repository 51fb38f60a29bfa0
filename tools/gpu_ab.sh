#!/bin/bash
# Interleaved A/B of one environment knob on the ResNet-50 training bench (GPU box).
#   tools/gpu_ab.sh VAR "VAL_A VAL_B ..." ROUNDS [bench args]
# AB_SCRIPT=tools/bench_inference.py (or any script printing the bench JSON line) A/Bs that bench instead.
# Runs bench.py once per value per round, values interleaved (A B A B ...) so box drift hits every arm alike, and
# prints "VAR=VAL ms_per_step" lines; each run bounded by its own timeout, the first failure ends the script.
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
var=$1; vals=$2; rounds=${3:-2}; shift 3
args=${*:-"--steps 20 --warmup 5"}
script=${AB_SCRIPT:-bench.py}
for r in $(seq 1 "$rounds"); do
  for v in $vals; do
    log=gpurun_out/ab_$(basename $script .py)_${var}_${v}_$r.log
    env "$var=$v" timeout -k 10 300 python -u $script $args > "$log" 2>&1 || { tail -20 "$log"; exit 1; }
    echo "$var=$v round $r $(tail -1 "$log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["config"].get("graph_vs_eager"))')"
  done
done
