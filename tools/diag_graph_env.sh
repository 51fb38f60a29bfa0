#!/bin/bash
# HIP-graph divergence probe: tools/diag_fork_graph.py variants under HIP runtime knobs, one process each.
#   bash tools/diag_graph_env.sh VARIANTS KNOB=VAL[,KNOB=VAL] ...   (first arg: variants, e.g. "B C")
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
vars=$1; shift
for cfg in "$@"; do
  envs=(); [ "$cfg" != "none" ] && IFS=',' read -ra envs <<< "$cfg"
  echo "## env: $cfg  variants: $vars" | tee -a gpurun_out/diag_graph_env.log
  env "${envs[@]}" timeout -k 10 240 python -u tools/diag_fork_graph.py $vars 2>&1 | grep -E "part|Error|error" \
    | tee -a gpurun_out/diag_graph_env.log; rc=$?
  [ $rc -eq 0 ] || exit $rc
done
