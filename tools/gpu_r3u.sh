set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
run() {  # name, graph, env...
  name=$1; g=$2; shift; shift
  env "$@" BIGDL_FORCE_COLLECTIVES=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 1 --steps 20 --warmup 5 --graph $g > gpurun_out/bench_$name.log 2>&1 || { tail -20 gpurun_out/bench_$name.log; exit 1; }
  echo "$name $(tail -1 gpurun_out/bench_$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"]["graph_vs_eager"], d["config"]["hip_graph"])')"
}
run fc_g1 1
run fc_auto -1
run fc_auto_ws0 -1 BIGDL_WGRAD_STREAM=0
