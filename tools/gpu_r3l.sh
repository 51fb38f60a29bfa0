set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "wgrad" --timeout 120 --timeout-method thread > gpurun_out/pytest_wg3.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_wg3.log
[ $rc -eq 0 ] || exit $rc
for g in 0 1 0 1; do
  BIGDL_WGRAD_G3=$g timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --graph 0 > gpurun_out/bench_wg3_$g.log 2>&1 || { tail -20 gpurun_out/bench_wg3_$g.log; exit 1; }
  echo "wg3=$g $(tail -1 gpurun_out/bench_wg3_$g.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"]["final_loss"])')"
done
timeout -k 10 500 python -u tools/bench_conv.py --no-miopen --iters 10 > gpurun_out/bench_conv_g4.log 2>&1; rc=$?
tail -1 gpurun_out/bench_conv_g4.log | cut -c1-300
exit $rc
