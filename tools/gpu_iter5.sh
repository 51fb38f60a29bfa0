# halo-tile 3x3 weight gradient: numerics, per-layer A/B against the split-K im2col kernels, training step
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "halo or wgrad" -x -q --timeout 120 --timeout-method thread > gpurun_out/t9a.log 2>&1; rc=$?; tail -5 gpurun_out/t9a.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/conv_variants.py --layers 2,10,16,22 --ops wgrad --variants "glds:halo=0;halo:halo=1" > gpurun_out/halo_ab.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/halo_ab.log
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/bench9.log 2>&1 || exit 1
tail -1 gpurun_out/bench9.log | cut -c1-200
timeout -k 10 300 python tools/diag_lm_aten.py > gpurun_out/lm_aten2.log 2>&1 || exit 1
grep -A 60 "GPU work" gpurun_out/lm_aten2.log | cut -c1-180
