export PYTHONPATH=$PWD
run() { tag=$1; shift; env "$@" timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bis_$tag.log 2>&1 || { tail -5 gpurun_out/bis_$tag.log; exit 1; }
  echo "$tag $(tail -1 gpurun_out/bis_$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"]["final_loss"], d["config"]["graph_vs_eager"])')"; }
run base BIGDL_X=0
run fill0 BIGDL_NATIVE_FILL=0
run base2 BIGDL_X=1
for v in 1 0; do
  BIGDL_WGRAD_P8=$v timeout -k 10 300 python -u tools/bench_lstm.py --steps 10 --warmup 3 --batch 128 > gpurun_out/r4i_lstm_$v.log 2>&1 || { tail -20 gpurun_out/r4i_lstm_$v.log; exit 1; }
  echo "LSTM WGRAD_P8=$v $(tail -1 gpurun_out/r4i_lstm_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["config"])')"
done
BIGDL_WGRAD_P8=1 timeout -k 10 300 python -u tools/bench_lstm.py --steps 10 --warmup 3 --batch 128 --graph 0 > gpurun_out/r4i_lstm_eager.log 2>&1 || exit 1
echo "LSTM eager $(tail -1 gpurun_out/r4i_lstm_eager.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["config"])')"
