# int8 streaming kernel tests + int8/bf16 inference benches, deterministic-mode cost, wgrad PMC on 3x3 layers
export PYTHONPATH=$PWD
timeout -k 10 800 python -u -m pytest tests/test_quantized_gpu.py tests/test_int8_graph_gpu.py tests/test_recurrent_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t7.log 2>&1; rc=$?; tail -4 gpurun_out/t7.log; [ $rc -eq 0 ] || exit $rc
for m in resnet50 inception_v3; do for md in int8 bf16; do
  timeout -k 10 300 python tools/bench_inference.py --model $m --mode $md > gpurun_out/inf_${m}_${md}.log 2>&1 || exit 1
  tail -1 gpurun_out/inf_${m}_${md}.log | cut -c1-300
done; done
for b in 128 256; do
  timeout -k 10 400 python tools/bench_lstm.py --batch $b > gpurun_out/lstm_b$b.log 2>&1 || exit 1
  tail -1 gpurun_out/lstm_b$b.log | cut -c1-250
done
timeout -k 10 300 python -c "
import sys; sys.path.insert(0, 'tools')
from det_check import run
for det in (False, True, False, True):
    _, ms = run(8, det, depth=50, batch=256, classes=1000, image=224, dataset='ImageNet')
    print('R50 det', det, round(ms, 2), 'ms/step', flush=True)
" > gpurun_out/det_r50.log 2>&1; cat gpurun_out/det_r50.log | grep R50
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/wpmc
for L in 16 22 10; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES -d gpurun_out/wpmc/p1_$L -o run -- python3 tools/conv_layer_run.py --idx $L --op wgrad --iters 10 > gpurun_out/wpmc/p1_$L.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR -d gpurun_out/wpmc/p2_$L -o run -- python3 tools/conv_layer_run.py --idx $L --op wgrad --iters 10 > gpurun_out/wpmc/p2_$L.log 2>&1 || exit 1
  python tools/pmc_dump.py gpurun_out/wpmc/p*_$L/run_results.db --match wgrad > gpurun_out/wpmc/pmc_$L.txt; cat gpurun_out/wpmc/pmc_$L.txt
done
