export PYTHONPATH=$PWD
bash tools/gpu_run.sh tests || exit 1
BIGDL_FORCE_COLLECTIVES=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 1 --steps 5 --warmup 3 > gpurun_out/trun.log 2>&1 || { tail -20 gpurun_out/trun.log; exit 1; }
tail -1 gpurun_out/trun.log | cut -c1-300
bash tools/gpu_run.sh dist prof || exit 1
timeout -k 10 300 python tools/bench_lstm.py --steps 10 --warmup 3 --batch 128 > gpurun_out/lstm_b128.log 2>&1 || { tail -20 gpurun_out/lstm_b128.log; exit 1; }
tail -1 gpurun_out/lstm_b128.log | cut -c1-300
(cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && rm -rf gpurun_out/lstmprof && \
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/lstmprof -o run -- python3 tools/bench_lstm.py --steps 2 --warmup 1 --batch 128 --graph 0 \
  > gpurun_out/lstm_prof.log 2>&1) || { tail -20 gpurun_out/lstm_prof.log; exit 1; }
