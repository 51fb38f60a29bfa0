# Short-K (two-stage, 4 workgroups per CU) variants: exactness / numerics tests, then the int8 A/B
# (tools/gpu_int8_ab.sh BIGDL_I8_SHORTK) and the bf16 training bench A/B (BIGDL_CONV_SHORTK) on one MI355X.
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "g4_kernel" > gpurun_out/sk_test.log 2>&1; rc=$?; tail -2 gpurun_out/sk_test.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_int8_ab.sh BIGDL_I8_SHORTK "0 1 2" || exit 1
for r in 1 2; do for v in 0 1; do
  BIGDL_CONV_SHORTK=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/sk_bench_${v}_$r.log 2>&1 || { tail -5 gpurun_out/sk_bench_${v}_$r.log; exit 1; }
  echo "BIGDL_CONV_SHORTK=$v run $r: $(tail -1 gpurun_out/sk_bench_${v}_$r.log | cut -c120-200)"
done; done
