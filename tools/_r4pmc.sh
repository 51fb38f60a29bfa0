export PYTHONPATH=$PWD
bash tools/gpu_run.sh pmc=SQ_WAVE_CYCLES,SQ_BUSY_CU_CYCLES,SQ_VALU_MFMA_BUSY_CYCLES,GRBM_GUI_ACTIVE,SQ_LDS_BANK_CONFLICT,SQ_INSTS_LDS pmc=FETCH_SIZE pmc=WRITE_SIZE || exit 1
(cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && rm -rf gpurun_out/lstmprof && \
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/lstmprof -o run -- python3 tools/bench_lstm.py --steps 3 --warmup 2 --batch 128 --graph 0 \
  > gpurun_out/lstm_prof.log 2>&1) || { tail -20 gpurun_out/lstm_prof.log; exit 1; }
echo done
