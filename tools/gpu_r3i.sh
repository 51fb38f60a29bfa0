set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest.log 2>&1; rc=$?
tail -8 gpurun_out/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1; rc=$?
tail -1 gpurun_out/bench.log | cut -c1-1200
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --via-optimizer > gpurun_out/bench_opt.log 2>&1; rc=$?
tail -1 gpurun_out/bench_opt.log | cut -c1-1200
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u tools/bench_data_pipeline.py > gpurun_out/data_pipeline.log 2>&1; rc=$?
tail -3 gpurun_out/data_pipeline.log
exit $rc
