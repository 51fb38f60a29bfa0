# PMC passes over the ResNet-50 training step (eager, 2 timed steps): MFMA busy and HBM bytes per kernel
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
ROOT=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
rm -rf gpurun_out/pmcs_1 gpurun_out/pmcs_2
timeout -s KILL 240 rocprofv3 --pmc SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES -d gpurun_out/pmcs_1 -o run -- python3 bench.py --steps 2 --warmup 2 --graph 0 > gpurun_out/pmcs_1.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcs_2 -o run -- python3 bench.py --steps 2 --warmup 2 --graph 0 > gpurun_out/pmcs_2.log 2>&1 || exit 1
python3 tools/pmc_table.py $(ls gpurun_out/pmcs_1/*/run_results.db gpurun_out/pmcs_1/run_results.db 2>/dev/null | head -1) $(ls gpurun_out/pmcs_2/*/run_results.db gpurun_out/pmcs_2/run_results.db 2>/dev/null | head -1) --top 20 > gpurun_out/pmc_step.txt
cat gpurun_out/pmc_step.txt
