set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_distributed_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_dist.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_dist.log
[ $rc -eq 0 ] || exit $rc
for g in 0 -1; do
  BIGDL_FORCE_COLLECTIVES=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 1 --steps 20 --warmup 5 --graph $g > gpurun_out/bench_fc$g.log 2>&1 || { tail -20 gpurun_out/bench_fc$g.log; exit 1; }
  echo "forced graph=$g $(tail -1 gpurun_out/bench_fc$g.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"]["graph_vs_eager"], d["config"]["final_loss"])')"
done
