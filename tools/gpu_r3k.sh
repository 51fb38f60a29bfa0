set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
for w in 1024 512 256 1024 512 256; do
  BIGDL_WGRAD_WGS=$w timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --graph 0 > gpurun_out/bench_wgs_$w.log 2>&1 || { tail -20 gpurun_out/bench_wgs_$w.log; exit 1; }
  echo "wgs=$w $(tail -1 gpurun_out/bench_wgs_$w.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"]["final_loss"])')"
done
