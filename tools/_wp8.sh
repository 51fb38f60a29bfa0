# wgrad P8 kernel: numerics, per-layer wgrad roofline on/off, bench A/B
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "wgrad" > gpurun_out/wp8_test.log 2>&1; rc=$?; tail -5 gpurun_out/wp8_test.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0; do
  BIGDL_WGRAD_P8=$v timeout -k 10 300 python -u tools/conv_roofline.py --iters 10 > gpurun_out/wp8_roof_$v.log 2>&1 || { tail -20 gpurun_out/wp8_roof_$v.log; exit 1; }
  echo "== WGRAD_P8=$v"; grep -i "wgrad\|total" gpurun_out/wp8_roof_$v.log | tail -25
done
bash tools/gpu_ab.sh BIGDL_WGRAD_P8 "1 0" 3
