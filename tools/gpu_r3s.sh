set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
for g in -1 0; do
  BIGDL_BENCH_TRACE=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --graph $g > gpurun_out/bench_s$g.log 2>&1 || { tail -20 gpurun_out/bench_s$g.log; exit 1; }
  echo "graph=$g $(tail -1 gpurun_out/bench_s$g.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"]["graph_vs_eager"])')"
  grep "bench trace" gpurun_out/bench_s$g.log | head -2
done
