set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for mode in int8 bf16; do
  rm -rf gpurun_out/prof_r50_$mode
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50_$mode -o run -- python3 tools/bench_inference.py --model resnet50 --mode $mode --steps 5 > gpurun_out/prof_r50_$mode.log 2>&1 || { tail -20 gpurun_out/prof_r50_$mode.log; exit 1; }
  tail -1 gpurun_out/prof_r50_$mode.log
done
