# stream-K P8 + GRU persistent + LSTM NT2 checks, SK A/B on deep-K layers, LM aten census, bench
export PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "s1_stream or p8_stream_k or p8_kernel or w8" -x -q --timeout 200 --timeout-method thread > gpurun_out/t8a.log 2>&1; rc=$?; tail -4 gpurun_out/t8a.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_recurrent_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t8b.log 2>&1; rc=$?; tail -4 gpurun_out/t8b.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/conv_variants.py --layers 12,15,16,17,18,20,21,22 --ops fwd,dgrad --variants "sk0:sk=0;sk1:sk=1" > gpurun_out/sk_ab.log 2>&1 || exit 1
cat gpurun_out/sk_ab.log
timeout -k 10 300 python tools/diag_lm_aten.py > gpurun_out/lm_aten.log 2>&1 || exit 1
tail -30 gpurun_out/lm_aten.log
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/bench8.log 2>&1 || exit 1
tail -1 gpurun_out/bench8.log
