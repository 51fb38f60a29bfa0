set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
for i in 1 2 3 4 5; do
  BIGDL_BENCH_TRACE=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 $EXTRA > gpurun_out/bench_s$i.log 2>&1 || { tail -20 gpurun_out/bench_s$i.log; exit 1; }
  echo "run $i $(tail -1 gpurun_out/bench_s$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"]["graph_vs_eager"])')"
  grep "gaps" gpurun_out/bench_s$i.log | cut -c1-400
done
