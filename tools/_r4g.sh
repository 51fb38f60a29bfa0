export PYTHONPATH=$PWD
mkdir -p gpurun_out/pmcw
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_recurrent_gpu.py -x -q --timeout 120 --timeout-method thread -k "wgrad_p8 or lstm or recurrent or rnn or embedding" > gpurun_out/r4g_test.log 2>&1; rc=$?; tail -3 gpurun_out/r4g_test.log; [ $rc -eq 0 ] || exit $rc
for v in 2 0; do BIGDL_WGRAD_P8=$v timeout -k 10 120 python -u tools/wgrad_p8_probe.py || exit 1; done
for v in 1 0; do
  BIGDL_WGRAD_P8=$v timeout -k 10 300 python -u tools/bench_lstm.py --steps 10 --warmup 3 --batch 128 > gpurun_out/r4g_lstm_$v.log 2>&1 || { tail -20 gpurun_out/r4g_lstm_$v.log; exit 1; }
  echo "WGRAD_P8=$v $(tail -1 gpurun_out/r4g_lstm_$v.log | cut -c1-200)"
done
(cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && rm -rf gpurun_out/lstmprof && \
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/lstmprof -o run -- python3 tools/bench_lstm.py --steps 2 --warmup 1 --batch 128 --graph 0 \
  > gpurun_out/lstm_prof.log 2>&1) || { tail -20 gpurun_out/lstm_prof.log; exit 1; }
echo done
timeout -k 10 300 python -u -m pytest tests/test_quantized_gpu.py tests/test_int8_graph_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4g_i8test.log 2>&1; rc=$?; tail -3 gpurun_out/r4g_i8test.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0; do for m in resnet50 inception_v3; do
  BIGDL_I8_P8=$v timeout -k 10 300 python -u tools/bench_inference.py --model $m --mode int8 > gpurun_out/r4g_inf_${m}_$v.log 2>&1 || { tail -20 gpurun_out/r4g_inf_${m}_$v.log; exit 1; }
  echo "I8_P8=$v $m $(tail -1 gpurun_out/r4g_inf_${m}_$v.log | cut -c1-220)"
done; done
for m in resnet50 inception_v3; do
  timeout -k 10 300 python -u tools/bench_inference.py --model $m --mode bf16 > gpurun_out/r4g_inf_${m}_bf16.log 2>&1 || { tail -20 gpurun_out/r4g_inf_${m}_bf16.log; exit 1; }
  echo "bf16 $m $(tail -1 gpurun_out/r4g_inf_${m}_bf16.log | cut -c1-220)"
done
