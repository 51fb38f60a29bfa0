# halo kernel with branch-free epilogues: numerics, ablation (no epilogue), per-layer A/B, step
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "halo or bn_fwd_bwd" -x -q --timeout 120 --timeout-method thread > gpurun_out/halo_t.log 2>&1; rc=$?; tail -5 gpurun_out/halo_t.log; [ $rc -eq 0 ] || exit $rc
BIGDL_CONV_HALO_ABL=1 timeout -k 10 200 python tools/conv_variants.py --layers 2,10,16,22 --ops fwd_nostats --variants "noepi:chalo=1" --rounds 3 > gpurun_out/halo_abl_1.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/halo_abl_1.log
timeout -k 10 300 python tools/conv_variants.py --layers 2,10,16,22 --ops fwd,fwd_nostats,dgrad_bn --variants "halo:chalo=1;im2col:chalo=0" > gpurun_out/halo_ab.log 2>&1 || { tail -20 gpurun_out/halo_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/halo_ab.log
for cfg in "BIGDL_CONV_HALO=1" "BIGDL_CONV_HALO=0" "BIGDL_CONV_HALO=1"; do
  env $cfg timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/bench_halo.log 2>&1 || { tail -20 gpurun_out/bench_halo.log; exit 1; }
  echo "$cfg $(tail -1 gpurun_out/bench_halo.log | cut -c1-200)"
done
