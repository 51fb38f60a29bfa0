set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
# one RCCL rank with every collective forced on (bucketed reduce-scatter / all-gather, segmented HIP graphs, side stream)
BIGDL_FORCE_COLLECTIVES=1 BIGDL_BENCH_TRACE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_forced.log 2>&1; rc=$?
tail -1 gpurun_out/bench_forced.log | cut -c1-900; grep "bench trace" gpurun_out/bench_forced.log | head -3
[ $rc -eq 0 ] || exit $rc
# two gloo ranks sharing the GPU (multi-rank rehearsal)
BIGDL_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 3 --warmup 2 --batch 64 > gpurun_out/dist.log 2>&1; rc=$?
tail -1 gpurun_out/dist.log | cut -c1-600
exit $rc
