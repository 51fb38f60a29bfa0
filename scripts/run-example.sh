#!/bin/bash
# Smoke-run the model zoo on synthetic data (reference run.example.sh): each family trains a few
# iterations through the Optimizer and reports throughput.
#   scripts/run-example.sh [model ...]      (default: lenet5 resnet autoencoder rnn)
set -euo pipefail
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)"
export PYTHONPATH="$HERE${PYTHONPATH:+:$PYTHONPATH}"
MODELS=("$@")
[ ${#MODELS[@]} -gt 0 ] || MODELS=(lenet5 resnet autoencoder rnn)
for m in "${MODELS[@]}"; do
  echo "== $m"
  python3 -m bigdl_amd.models.cli perf --model "$m" --batchSize 32 --iteration 3
done
