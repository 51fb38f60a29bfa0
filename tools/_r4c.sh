# LSTM kernel table (persistent path), wgrad P8 rule A/B, GPU test tier
export PYTHONPATH=$PWD
mkdir -p gpurun_out
(cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && rm -rf gpurun_out/lstmprof && \
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/lstmprof -o run -- python3 tools/bench_lstm.py --steps 2 --warmup 1 --batch 128 --graph 0 \
  > gpurun_out/lstm_prof.log 2>&1) || { tail -20 gpurun_out/lstm_prof.log; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "wgrad" tests/test_optimizer_graph_gpu.py -s > gpurun_out/r4c_test.log 2>&1; rc=$?; tail -3 gpurun_out/r4c_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/bench_conv_stats.py > gpurun_out/conv_stats.log 2>&1 || { tail -5 gpurun_out/conv_stats.log; exit 1; }
cat gpurun_out/conv_stats.log
bash tools/gpu_ab.sh BIGDL_WGRAD_P8 "1 0" 3
for v in 1 0; do
  BIGDL_G4_ABN=$v timeout -k 10 300 python -u tools/conv_roofline.py --iters 10 > gpurun_out/abn_roof_$v.log 2>&1 || { tail -20 gpurun_out/abn_roof_$v.log; exit 1; }
  echo "== G4_ABN=$v"; grep "fwd:\|dgrad:" gpurun_out/abn_roof_$v.log
done
