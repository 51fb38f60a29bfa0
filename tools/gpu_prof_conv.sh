#!/bin/bash
# Kernel-time profile of the ResNet-50 training step + PMC counters of the conv kernels on representative shapes.
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace -o run -- python3 bench.py --steps 5 --warmup 3 --graph 0 > gpurun_out/prof/bench.log 2>&1 || { echo "trace run failed"; tail -20 gpurun_out/prof/bench.log; exit 1; }
tail -1 gpurun_out/prof/bench.log
timeout -k 10 600 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d gpurun_out/prof/pmc1 -o pmc -- python3 tools/bench_conv.py --iters 3 --only 2,13,16,22 --no-miopen > gpurun_out/prof/pmc1.log 2>&1 || { echo "pmc run failed"; tail -20 gpurun_out/prof/pmc1.log; exit 2; }
timeout -k 10 600 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_ANY -d gpurun_out/prof/pmc2 -o pmc -- python3 tools/bench_conv.py --iters 3 --only 2,13,16,22 --no-miopen > gpurun_out/prof/pmc2.log 2>&1 || { echo "pmc2 run failed"; tail -20 gpurun_out/prof/pmc2.log; exit 3; }
find gpurun_out/prof -name "*.csv" | head -20
