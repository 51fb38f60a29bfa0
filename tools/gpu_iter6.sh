# halo wgrad after the vmcnt fix: numerics, per-layer A/B, PMC of layer 16, training step
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "halo or wgrad" -x -q --timeout 120 --timeout-method thread > gpurun_out/t10a.log 2>&1; rc=$?; tail -3 gpurun_out/t10a.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/conv_variants.py --layers 2,10,16,22 --ops wgrad --variants "glds:halo=0;halo:halo=1" > gpurun_out/halo_ab2.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/halo_ab2.log
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/bench10.log 2>&1 || exit 1
tail -1 gpurun_out/bench10.log | cut -c1-200
BIGDL_WGRAD_HALO=0 timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/bench10_off.log 2>&1 || exit 1
tail -1 gpurun_out/bench10_off.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/hpmc
for L in 16 2; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES -d gpurun_out/hpmc/p1_$L -o run -- python3 tools/conv_layer_run.py --idx $L --op wgrad --iters 10 > gpurun_out/hpmc/p1_$L.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR -d gpurun_out/hpmc/p2_$L -o run -- python3 tools/conv_layer_run.py --idx $L --op wgrad --iters 10 > gpurun_out/hpmc/p2_$L.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d gpurun_out/hpmc/kt_$L -o run -- python3 tools/conv_layer_run.py --idx $L --op wgrad --iters 10 > gpurun_out/hpmc/kt_$L.log 2>&1 || exit 1
  python tools/pmc_dump.py gpurun_out/hpmc/p*_$L/run_results.db > gpurun_out/hpmc/pmc_$L.txt; cat gpurun_out/hpmc/pmc_$L.txt | head -40
done
