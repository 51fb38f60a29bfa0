# LSTM kernel table (persistent path), wgrad P8 rule A/B, GPU test tier
export PYTHONPATH=$PWD
mkdir -p gpurun_out
(cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && rm -rf gpurun_out/lstmprof && \
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/lstmprof -o run -- python3 tools/bench_lstm.py --steps 2 --warmup 1 --batch 128 --graph 0 \
  > gpurun_out/lstm_prof.log 2>&1) || { tail -20 gpurun_out/lstm_prof.log; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "wgrad" > gpurun_out/r4c_test.log 2>&1; rc=$?; tail -3 gpurun_out/r4c_test.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab.sh BIGDL_WGRAD_P8 "1 0" 3
