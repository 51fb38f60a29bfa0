# rocprofv3 kernel tables of the int8 and bf16 inference steps (tools/bench_inference.py)
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
M=${1:-resnet50}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for mode in int8 bf16; do
  rm -rf gpurun_out/prof_${M}_$mode
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${M}_$mode -o run -- python3 tools/bench_inference.py --model $M --mode $mode --steps 5 > gpurun_out/prof_${M}_$mode.log 2>&1 || { tail -20 gpurun_out/prof_${M}_$mode.log; exit 1; }
  tail -1 gpurun_out/prof_${M}_$mode.log | cut -c1-200
done
