export PYTHONPATH=$PWD
for i in 1 2 3; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$i.log 2>&1 || { tail -20 gpurun_out/bench_$i.log; exit 1; }
tail -1 gpurun_out/bench_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench", d["ms_per_step"], d["value"], d["config"]["final_loss"], d["config"]["graph_vs_eager"])'
done
BIGDL_BENCH_TRACE=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --graph 0 > gpurun_out/bench_tr.log 2>&1 || { tail -20 gpurun_out/bench_tr.log; exit 1; }
tail -3 gpurun_out/bench_tr.log | cut -c1-300
