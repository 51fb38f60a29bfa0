# Single-layer study of the streaming-bound 1x1 convs: interleaved timing A/B (tools/conv_variants.py) and PMC passes
# of one layer (tools/conv_layer_run.py). Args: LAYER OP VARIANTS
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out/study
L=${1:-3}; OP=${2:-fwd}; V=${3:-"base:"}
timeout -k 10 300 python -u tools/conv_variants.py --layers 1,3,4,7,13,15 --variants "$V" > gpurun_out/study/variants.log 2>&1 || exit 1
cat gpurun_out/study/variants.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {  # tag counters...
  tag=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d gpurun_out/study/$tag -o run -- python3 tools/conv_layer_run.py --idx $L --op $OP --iters 10 > gpurun_out/study/$tag.log 2>&1
}
run p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS || exit 1
run p2 SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU || exit 1
run p3 FETCH_SIZE GRBM_GUI_ACTIVE || exit 1
run p4 WRITE_SIZE TCC_HIT_sum TCC_MISS_sum || exit 1

python tools/pmc_dump.py gpurun_out/study/p*/run_results.db --match conv > gpurun_out/study/pmc.txt
cat gpurun_out/study/pmc.txt
