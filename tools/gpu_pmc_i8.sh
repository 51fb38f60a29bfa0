# PMC passes over one int8 roofline layer (tools/int8_roofline.py --only IDX: int8 conv then bf16 conv of that shape)
export PYTHONPATH=$PWD
idx=${1:-3}
mkdir -p gpurun_out/pmci8
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {  # tag counters...
  tag=$1; shift
  timeout -s KILL 60 rocprofv3 --pmc "$@" -d gpurun_out/pmci8/$tag -o run --output-format csv -- python3 tools/int8_roofline.py --only $idx --iters 10 > gpurun_out/pmci8/$tag.log 2>&1
}
run p1_$idx SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS || exit 1
run p2_$idx FETCH_SIZE || exit 1
run p3_$idx WRITE_SIZE || exit 1
run p4_$idx SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM_WR SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE || exit 1
echo pmc-done
