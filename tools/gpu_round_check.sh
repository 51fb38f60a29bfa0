export PYTHONPATH=$PWD
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest.log 2>&1; rc=$?; tail -5 gpurun_out/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_run.sh smoke || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-400
BIGDL_FORCE_COLLECTIVES=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 1 --steps 5 --warmup 3 > gpurun_out/trun.log 2>&1 || { tail -20 gpurun_out/trun.log; exit 1; }
tail -1 gpurun_out/trun.log | cut -c1-300
bash tools/gpu_run.sh dist prof || exit 1
echo round-check-done
