# wgrad P8 + persistent LSTM: numerics, LSTM bench seq on/off, wgrad roofline/bench A/B
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_recurrent_gpu.py -x -q --timeout 120 --timeout-method thread -k "wgrad or lstm or recurrent or gru" > gpurun_out/r4b_test.log 2>&1; rc=$?; tail -8 gpurun_out/r4b_test.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0; do
  BIGDL_LSTM_SEQ=$v timeout -k 10 300 python -u tools/bench_lstm.py --steps 10 --warmup 3 --batch 128 > gpurun_out/r4b_lstm_$v.log 2>&1 || { tail -20 gpurun_out/r4b_lstm_$v.log; exit 1; }
  echo "LSTM_SEQ=$v $(tail -1 gpurun_out/r4b_lstm_$v.log | cut -c1-260)"
done
for v in 1 0; do
  BIGDL_WGRAD_P8=$v timeout -k 10 300 python -u tools/conv_roofline.py --iters 10 > gpurun_out/r4b_roof_$v.log 2>&1 || { tail -20 gpurun_out/r4b_roof_$v.log; exit 1; }
  echo "== WGRAD_P8=$v"; grep -i "total" gpurun_out/r4b_roof_$v.log | tail -5
done
bash tools/gpu_ab.sh BIGDL_WGRAD_P8 "1 0" 2
