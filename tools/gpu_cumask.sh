# weight-gradient side stream restricted to a CU subset (BIGDL_WGRAD_CUMASK); "first:256" = an external stream on all CUs
export PYTHONPATH=$PWD
for m in "" "first:256" "stride:2" "" "first:256"; do
  BIGDL_WGRAD_CUMASK=$m timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/bench_cm.log 2>&1 || { tail -20 gpurun_out/bench_cm.log; exit 1; }
  echo "mask=[$m] $(tail -1 gpurun_out/bench_cm.log | grep -o '"ms_per_step": [0-9.]*')  $(tail -1 gpurun_out/bench_cm.log | grep -o '"graph_vs_eager": {[^}]*}')"
done
