export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "maxpool" -x -q --timeout 120 --timeout-method thread > gpurun_out/pool_t.log 2>&1; rc=$?; tail -3 gpurun_out/pool_t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python - <<'PY'
import torch, time, os, sys
sys.path.insert(0, os.getcwd())
from bigdl_amd.ops import pool, native
x = torch.randn(256, 64, 112, 112, device="cuda").to(torch.bfloat16, memory_format=torch.channels_last)
y, idx = pool.maxpool_fwd_gpu(x, 3, 3, 2, 2, 1, 1)
gy = torch.randn_like(y)
for name in ("k3s2", "gather"):
    if name == "gather":
        os.environ["BIGDL_POOL_BWD_K3S2"] = "0"
    for _ in range(3): dx = pool.maxpool_bwd_gpu(gy, idx, x.shape, 3, 3, 2, 2, 1, 1)
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(20): dx = pool.maxpool_bwd_gpu(gy, idx, x.shape, 3, 3, 2, 2, 1, 1)
    torch.cuda.synchronize(); print(name, "maxpool bwd us", (time.perf_counter() - t) / 20 * 1e6)
PY
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/bench_pool.log 2>&1 || { tail -20 gpurun_out/bench_pool.log; exit 1; }
  echo "bench $(tail -1 gpurun_out/bench_pool.log | grep -o '"ms_per_step": [0-9.]*')"
done
