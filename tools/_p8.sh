export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "p8 or w8 or g4_kernel or fwd_dgrad_wgrad or nt_variants" > gpurun_out/p8_test.log 2>&1; rc=$?; tail -5 gpurun_out/p8_test.log; [ $rc -eq 0 ] || exit $rc
for cfg in BIGDL_CONV_P8=1 BIGDL_CONV_P8=0; do
  env $cfg timeout -k 10 120 python -u tools/gemm_ceiling.py 2>&1 | grep TF || exit 1
done
