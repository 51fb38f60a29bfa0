export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "p8 or w8 or fwd_dgrad_wgrad" > gpurun_out/p8kt_test.log 2>&1; rc=$?; tail -3 gpurun_out/p8kt_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_lstm.py --steps 10 --warmup 3 --batch 128 > gpurun_out/p8kt_lstm.log 2>&1 || { tail -5 gpurun_out/p8kt_lstm.log; exit 1; }
tail -1 gpurun_out/p8kt_lstm.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("lstm", d["ms_per_step"], d["value"], d["config"]["final_loss"])'
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/p8kt_bench.log 2>&1 || exit 1
tail -1 gpurun_out/p8kt_bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench", d["ms_per_step"], d["value"], d["config"]["final_loss"])'
