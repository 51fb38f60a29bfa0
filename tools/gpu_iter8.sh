# stem overlapping-window forward + halo wgrad in the training step
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/test_conv_family_gpu.py -k "pair" -x -q --timeout 120 --timeout-method thread > gpurun_out/t12a.log 2>&1; rc=$?; tail -3 gpurun_out/t12a.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_stem.py > gpurun_out/stem1.log 2>&1 || exit 1
tail -1 gpurun_out/stem1.log
for cfg in "BIGDL_WGRAD_HALO=1" "BIGDL_WGRAD_HALO=0" "BIGDL_WGRAD_HALO_LDS=80" "BIGDL_STEM_WINDOW=0"; do
  env $cfg timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/bench12.log 2>&1 || exit 1
  echo "$cfg $(tail -1 gpurun_out/bench12.log | cut -c1-200)"
done
