export PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest tests/test_recurrent_gpu.py tests/test_optimizer_graph_gpu.py tests/test_distributed_gpu.py tests/test_straggler_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4j_test.log 2>&1; rc=$?; tail -3 gpurun_out/r4j_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench", d["ms_per_step"], d["value"], d["config"]["final_loss"], d["config"]["graph_vs_eager"])'
timeout -k 10 300 python -u tools/bench_lstm.py --steps 10 --warmup 3 --batch 128 > gpurun_out/lstm_b128.log 2>&1 || { tail -20 gpurun_out/lstm_b128.log; exit 1; }
tail -1 gpurun_out/lstm_b128.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("lstm", d["ms_per_step"], d["value"], d["config"])'
(cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && rm -rf gpurun_out/lstmprof && \
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/lstmprof -o run -- python3 tools/bench_lstm.py --steps 3 --warmup 2 --batch 128 --graph 0 \
  > gpurun_out/lstm_prof.log 2>&1) || { tail -20 gpurun_out/lstm_prof.log; exit 1; }
echo done
