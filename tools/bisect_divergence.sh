# ResNet-50 training divergence bisection: final_loss under toggles (short runs)
export PYTHONPATH=$PWD
run() { tag=$1; shift; env "$@" timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bis_$tag.log 2>&1 || { tail -5 gpurun_out/bis_$tag.log; exit 1; }
  echo "$tag $(tail -1 gpurun_out/bis_$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"]["final_loss"], d["config"]["graph_vs_eager"])')"; }
run base BIGDL_X=0
run fill0 BIGDL_NATIVE_FILL=0
run fill6 BIGDL_NATIVE_FILL=6
run fill5 BIGDL_NATIVE_FILL=5
run fill3 BIGDL_NATIVE_FILL=3
graph0() { timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --graph 0 > gpurun_out/bis_graph0.log 2>&1 || exit 1; echo "graph0 $(tail -1 gpurun_out/bis_graph0.log | cut -c1-80) loss $(tail -1 gpurun_out/bis_graph0.log | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['config']['final_loss'])")"; }; graph0
run p8w0 BIGDL_WGRAD_P8=0 BIGDL_CONV_P8=0
