export PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "bn or stats or halo or s1" -x -q --timeout 120 --timeout-method thread > gpurun_out/b3_t.log 2>&1; rc=$?; tail -2 gpurun_out/b3_t.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/b3.log 2>&1 || { tail -20 gpurun_out/b3.log; exit 1; }
  echo "run $i $(tail -1 gpurun_out/b3.log | grep -o '"ms_per_step": [0-9.]*')"
done
