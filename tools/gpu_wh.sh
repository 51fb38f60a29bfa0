export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "halo" -x -q --timeout 120 --timeout-method thread > gpurun_out/halo_t.log 2>&1; rc=$?; tail -3 gpurun_out/halo_t.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for cfg in "BIGDL_WGRAD_HALO=1" "BIGDL_WGRAD_HALO=0"; do
    env $cfg timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/ab2.log 2>&1 || { tail -20 gpurun_out/ab2.log; exit 1; }
    echo "$cfg round $i $(tail -1 gpurun_out/ab2.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
