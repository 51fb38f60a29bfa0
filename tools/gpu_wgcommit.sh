# workgroup-level statistics commit in nt_epilogue_lds: kernel numerics, stem + conv layer timings, training step
export PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_conv_family_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/wgc_t.log 2>&1; rc=$?; tail -5 gpurun_out/wgc_t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_stem.py > gpurun_out/stem.log 2>&1 || exit 1
tail -1 gpurun_out/stem.log
timeout -k 10 300 python tools/conv_variants.py --layers 1,3,4,5,7,9,11,13 --ops fwd,fwd_nostats,dgrad_bn --variants "base:" > gpurun_out/wgc_layers.log 2>&1 || { tail -20 gpurun_out/wgc_layers.log; exit 1; }
grep -v amdgpu.ids gpurun_out/wgc_layers.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/bench_wgc.log 2>&1 || { tail -20 gpurun_out/bench_wgc.log; exit 1; }
  echo "bench $(tail -1 gpurun_out/bench_wgc.log | grep -o '"ms_per_step": [0-9.]*')"
done
