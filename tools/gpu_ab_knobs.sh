#!/bin/bash
# Interleaved A/B of several env settings on the training bench: gpu_ab_knobs.sh "ENV1=a,ENV2=b" "none" ... (2 rounds)
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
for i in 1 2; do
  for cfg in "$@"; do
    envs=(); [ "$cfg" != "none" ] && IFS=',' read -ra envs <<< "$cfg"
    env "${envs[@]}" timeout -k 10 240 python bench.py --steps 30 --warmup 10 > gpurun_out/knob.log 2>&1 || exit 1
    echo "$cfg round $i $(python -c "import json;d=json.loads(open('gpurun_out/knob.log').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['value'])")"
  done
done
