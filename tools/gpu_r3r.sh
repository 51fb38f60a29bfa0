set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
python3 -c "import torch; print('priority range', torch.cuda.Stream.priority_range())"
for p in 0 -1 0 -1; do
  BIGDL_MAIN_PRIO=$p timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --graph 0 > gpurun_out/bench_prio$p.log 2>&1 || { tail -20 gpurun_out/bench_prio$p.log; exit 1; }
  echo "prio=$p $(tail -1 gpurun_out/bench_prio$p.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"]["final_loss"])')"
done
