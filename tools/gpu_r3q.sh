set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q -k "bn or batch or resnet" --timeout 120 --timeout-method thread > gpurun_out/pytest_q.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_q.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_q$i.log 2>&1 || { tail -20 gpurun_out/bench_q$i.log; exit 1; }
  echo "run $i $(tail -1 gpurun_out/bench_q$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"]["graph_vs_eager"], d["config"]["final_loss"])')"
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 3 --graph 0 > gpurun_out/prof_bench.log 2>&1; rc=$?
exit $rc
