export PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest tests/test_conv_family_gpu.py tests/test_models_gpu.py -k "stem or pair or bottleneck" -x -q --timeout 120 --timeout-method thread > gpurun_out/madd_t.log 2>&1; rc=$?; tail -3 gpurun_out/madd_t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_stem.py > gpurun_out/stem.log 2>&1 || exit 1
tail -1 gpurun_out/stem.log
for i in 1 2; do
  for cfg in "BIGDL_STEM_WGRAD=1" "BIGDL_STEM_WGRAD=0" "BIGDL_MASKED_ADDEND=1"; do
    env $cfg timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/ab2.log 2>&1 || { tail -20 gpurun_out/ab2.log; exit 1; }
    echo "$cfg round $i $(tail -1 gpurun_out/ab2.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
