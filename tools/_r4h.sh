export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "wgrad" > gpurun_out/r4h_test.log 2>&1; rc=$?; tail -2 gpurun_out/r4h_test.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0; do BIGDL_WGRAD_P8=$v timeout -k 10 120 python -u tools/wgrad_p8_probe.py || exit 1; done
for v in 1 0; do
  BIGDL_WGRAD_P8=$v timeout -k 10 300 python -u tools/bench_lstm.py --steps 10 --warmup 3 --batch 128 > gpurun_out/r4h_lstm_$v.log 2>&1 || { tail -20 gpurun_out/r4h_lstm_$v.log; exit 1; }
  echo "WGRAD_P8=$v $(tail -1 gpurun_out/r4h_lstm_$v.log | cut -c1-200)"
done
(cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && rm -rf gpurun_out/lstmprof && \
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/lstmprof -o run -- python3 tools/bench_lstm.py --steps 2 --warmup 1 --batch 128 --graph 0 \
  > gpurun_out/lstm_prof.log 2>&1) || { tail -20 gpurun_out/lstm_prof.log; exit 1; }
bash tools/gpu_ab.sh BIGDL_WGRAD_P8 "1 0" 2
bash tools/gpu_run.sh prof || exit 1
echo done
