#!/bin/bash
# Inference step kernel table (tools/bench_inference.py under rocprofv3 --kernel-trace --stats): gpu_inf_prof6.sh MODEL MODE
set -o pipefail
export PYTHONPATH=$PWD
ROOT=$PWD
mkdir -p gpurun_out
M=${1:-inception_v3}; MODE=${2:-int8}
(cd /tmp && export TMPDIR=/tmp && cd "$ROOT" && rm -rf gpurun_out/prof_inf && \
  timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/prof_inf -o run -- python3 tools/bench_inference.py \
  --model $M --mode $MODE --steps 5 > gpurun_out/prof_inf.log 2>&1) || { tail -20 gpurun_out/prof_inf.log; exit 1; }
db=$(ls gpurun_out/prof_inf/*/run_results.db gpurun_out/prof_inf/run_results.db 2>/dev/null | head -1)
[ -n "$db" ] || { echo "no rocpd database"; ls -R gpurun_out/prof_inf | head; exit 1; }
python tools/rocpd_summary.py kernels "$db" ${MARK:-quantize_wim2col_f32} ${SKIP:-3} ${PER:-5} > gpurun_out/inf_${M}_${MODE}_kernels.txt || exit 1
rm -rf gpurun_out/prof_inf
head -30 gpurun_out/inf_${M}_${MODE}_kernels.txt | cut -c1-160
