# P8 weight-gradient kernel on GEMM-shaped problems: timing on/off + PMC passes
export PYTHONPATH=$PWD
mkdir -p gpurun_out/pmcw
for v in 2 0; do BIGDL_WGRAD_P8=$v timeout -k 10 120 python -u tools/wgrad_p8_probe.py || exit 1; done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() { tag=$1; shift; BIGDL_WGRAD_P8=2 timeout -s KILL 90 rocprofv3 --pmc "$@" -d gpurun_out/pmcw/$tag -o run --output-format csv -- python3 tools/wgrad_p8_probe.py --shapes 32768x4096x1024 --iters 3 > gpurun_out/pmcw/$tag.log 2>&1 || { tail -5 gpurun_out/pmcw/$tag.log; exit 1; }; }
run p1 SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY GRBM_GUI_ACTIVE
run p2 FETCH_SIZE
run p3 SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY SQ_INSTS_VMEM
echo pmc-done
