# Per-step kernel table + stream overlap of the ResNet-50 training bench under rocprofv3 --kernel-trace (eager).
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
ROOT=$PWD
(cd /tmp && export TMPDIR=/tmp && cd "$ROOT" && rm -rf gpurun_out/prof && \
  timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 3 --graph 0 \
  > gpurun_out/prof_bench.log 2>&1) || exit 1
db=$(ls gpurun_out/prof/*/run_results.db gpurun_out/prof/run_results.db 2>/dev/null | head -1)
python tools/rocpd_summary.py kernels "$db" sgd4 2 5 > gpurun_out/prof_kernels.txt && cat gpurun_out/prof_kernels.txt | head -40
python tools/rocpd_streams.py "$db" sgd4 2 5 > gpurun_out/prof_streams.txt; cat gpurun_out/prof_streams.txt | head -20
