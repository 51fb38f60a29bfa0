set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
run() {  # name, env...
  name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 10 --warmup 5 --graph 0 > gpurun_out/bench_$name.log 2>&1 || { tail -20 gpurun_out/bench_$name.log; exit 1; }
  echo "$name $(tail -1 gpurun_out/bench_$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"]["final_loss"])')"
}
run ws1 BIGDL_WGRAD_STREAM=1
run ws2 BIGDL_WGRAD_STREAM=1 BIGDL_WGRAD_STREAMS=2
run ws3 BIGDL_WGRAD_STREAM=1 BIGDL_WGRAD_STREAMS=3
run ws1_hi BIGDL_WGRAD_STREAM=1 BIGDL_WGRAD_PRIO=-1
run ws2_hi BIGDL_WGRAD_STREAM=1 BIGDL_WGRAD_STREAMS=2 BIGDL_WGRAD_PRIO=-1
