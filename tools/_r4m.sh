export PYTHONPATH=$PWD
timeout -k 10 300 python -u tools/diag_cycles.py > gpurun_out/cycles.log 2>&1 || { tail -20 gpurun_out/cycles.log; exit 1; }
head -3 gpurun_out/cycles.log
for i in 1 2 3; do
BIGDL_BENCH_TRACE=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/benchtr_$i.log 2>&1 || { tail -20 gpurun_out/benchtr_$i.log; exit 1; }
echo "run $i $(tail -1 gpurun_out/benchtr_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"]["final_loss"], d["config"]["graph_vs_eager"])')"
grep "GiB after" gpurun_out/benchtr_$i.log | cut -c1-500
done
timeout -k 10 600 python -u -m pytest tests/test_models_gpu.py tests/test_graph_fusion_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4m_test.log 2>&1; rc=$?; tail -3 gpurun_out/r4m_test.log; exit $rc
