# halo wgrad: buffer-load DMA, parallel reduce, LDS budget 160 vs 80 (isolated and in the training step)
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "halo or wgrad" -x -q --timeout 120 --timeout-method thread > gpurun_out/t11a.log 2>&1; rc=$?; tail -3 gpurun_out/t11a.log; [ $rc -eq 0 ] || exit $rc
BIGDL_WGRAD_HALO_LDS=80 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "halo" -x -q --timeout 120 --timeout-method thread > gpurun_out/t11b.log 2>&1; rc=$?; tail -3 gpurun_out/t11b.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/conv_variants.py --layers 2,10,16,22 --ops wgrad --variants "glds:halo=0;halo:halo=1" > gpurun_out/halo_ab3.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/halo_ab3.log
BIGDL_WGRAD_HALO_LDS=80 timeout -k 10 300 python tools/conv_variants.py --layers 2,10,16,22 --ops wgrad --variants "glds:halo=0;halo80:halo=1" > gpurun_out/halo_ab3_80.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/halo_ab3_80.log
for cfg in "BIGDL_WGRAD_HALO=1" "BIGDL_WGRAD_HALO=0" "BIGDL_WGRAD_HALO_LDS=80"; do
  env $cfg timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/bench11.log 2>&1 || exit 1
  echo "$cfg $(tail -1 gpurun_out/bench11.log | cut -c1-200)"
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d gpurun_out/hpmc/kt2 -o run -- python3 tools/conv_layer_run.py --idx 2 --op wgrad --iters 10 > gpurun_out/hpmc/kt2.log 2>&1 || exit 1
find gpurun_out/hpmc/kt2 -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-150 | head -8
timeout -k 10 300 python -u -m pytest tests/test_conv_family_gpu.py -k "pair" -x -q --timeout 120 --timeout-method thread > gpurun_out/t11c.log 2>&1; rc=$?; tail -3 gpurun_out/t11c.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_stem.py > gpurun_out/stem1.log 2>&1 || exit 1
tail -2 gpurun_out/stem1.log
