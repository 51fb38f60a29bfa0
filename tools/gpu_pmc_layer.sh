# PMC passes over single conv layers, old kernels vs the 256x256 kernel (BIGDL_CONV_W8)
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out/pmcl
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rocprofv3 -L > gpurun_out/pmcl/counters.txt 2>&1 || true
run() {  # tag w8 idx counters...
  tag=$1; w8=$2; idx=$3; shift 3
  BIGDL_CONV_W8=$w8 timeout -s KILL 90 rocprofv3 --pmc "$@" -d gpurun_out/pmcl/$tag -o run --output-format csv -- python3 tools/conv_layer_run.py --idx $idx --iters 10 > gpurun_out/pmcl/$tag.log 2>&1
}
for idx in 17 16; do
 for w8 in 0 1; do
  run p1_${idx}_$w8 $w8 $idx SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE || exit 1
  run p2_${idx}_$w8 $w8 $idx FETCH_SIZE || exit 1
  run p3_${idx}_$w8 $w8 $idx TCC_HIT_sum TCC_MISS_sum || exit 1
 done
done
echo pmc-done
