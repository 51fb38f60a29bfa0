# LSTM dropout native path (numerics vs masked fp32 reference), recurrent suite, LM aten census
export PYTHONPATH=$PWD
timeout -k 10 400 python -u -m pytest tests/test_recurrent_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t13a.log 2>&1; rc=$?; tail -5 gpurun_out/t13a.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/diag_lm_aten.py > gpurun_out/lm_aten3.log 2>&1 || exit 1
grep -A 80 "GPU work" gpurun_out/lm_aten3.log | cut -c1-200
for b in 128 256; do
  timeout -k 10 400 python tools/bench_lstm.py --batch $b > gpurun_out/lstm_b$b.log 2>&1 || exit 1
  tail -1 gpurun_out/lstm_b$b.log | cut -c1-250
done
