set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_graph_fusion_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_f.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_f.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 5 --graph-model > gpurun_out/bench_graphmodel.log 2>&1; rc=$?
tail -3 gpurun_out/bench_graphmodel.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 5 > gpurun_out/bench_seq.log 2>&1; rc=$?
tail -3 gpurun_out/bench_seq.log
exit $rc
