export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/test_conv_family_gpu.py -k "stem or pair" -x -q --timeout 120 --timeout-method thread > gpurun_out/stem_t.log 2>&1; rc=$?; tail -3 gpurun_out/stem_t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_stem.py > gpurun_out/stem.log 2>&1 || exit 1
tail -1 gpurun_out/stem.log
BIGDL_STEM_FWD=0 timeout -k 10 300 python tools/bench_stem.py > gpurun_out/stem0.log 2>&1 || exit 1
echo "off: $(tail -1 gpurun_out/stem0.log)"
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/bench_stem.log 2>&1 || { tail -20 gpurun_out/bench_stem.log; exit 1; }
  echo "bench $(tail -1 gpurun_out/bench_stem.log | grep -o '"ms_per_step": [0-9.]*')"
done
