export PYTHONPATH=$PWD
mkdir -p gpurun_out/pmcw
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "wgrad_p8" > gpurun_out/r4f_test.log 2>&1; rc=$?; tail -2 gpurun_out/r4f_test.log; [ $rc -eq 0 ] || exit $rc
for v in 2 0; do BIGDL_WGRAD_P8=$v timeout -k 10 120 python -u tools/wgrad_p8_probe.py || exit 1; done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
BIGDL_WGRAD_P8=2 timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmcw/q1 -o run --output-format csv -- python3 tools/wgrad_p8_probe.py --shapes 32768x4096x1024 --iters 3 > gpurun_out/pmcw/q1.log 2>&1 || exit 1
echo done
