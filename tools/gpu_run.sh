#!/bin/bash
# One parameterised GPU-box driver (replaces the round-1 single-use gpu_*.sh scripts).
#   tools/gpu_run.sh STEP [STEP ...]
# Steps (each bounded by its own timeout, chained: the first failure ends the call):
#   tests[=PATTERN]   pytest -m gpu (optionally -k PATTERN)       -> gpurun_out/pytest.log
#   smoke             __graft_entry__.smoke()                     -> gpurun_out/smoke.log
#   bench[=ARGS]      python bench.py ARGS (default --steps 20 --warmup 5) -> gpurun_out/bench.log
#   prof[=ARGS]       rocprofv3 --kernel-trace --stats of bench.py (eager) -> gpurun_out/prof/
#   pmc=COUNTERS      rocprofv3 --pmc COUNTERS of bench.py (one pass)      -> gpurun_out/pmc_N/
#   py=SCRIPT[:ARGS]  python SCRIPT ARGS                           -> gpurun_out/<script>.log
#   dist[=ARGS]       2 ranks of bench.py on the one GPU over gloo (multi-rank rehearsal) -> gpurun_out/dist.log
set -o pipefail
export PYTHONPATH=$PWD
ROOT=$PWD
mkdir -p gpurun_out
npmc=0
for s in "$@"; do
  key=${s%%=*}; val=""; [ "$key" != "$s" ] && val=${s#*=}
  case $key in
    tests)
      k=(); [ -n "$val" ] && k=(-k "$val")
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "${k[@]}" \
        > gpurun_out/pytest.log 2>&1; rc=$?
      tail -15 gpurun_out/pytest.log; [ $rc -eq 0 ] || exit $rc ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
      tail -3 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc ;;
    bench)
      a=${val:-"--steps 20 --warmup 5"}
      timeout -k 10 600 python bench.py $a > gpurun_out/bench.log 2>&1; rc=$?
      tail -2 gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc ;;
    prof)
      a=${val:-"--steps 5 --warmup 3 --graph 0"}
      (cd /tmp && export TMPDIR=/tmp && cd "$ROOT" && rm -rf gpurun_out/prof && \
        timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py $a \
        > gpurun_out/prof_bench.log 2>&1); rc=$?
      tail -2 gpurun_out/prof_bench.log; [ $rc -eq 0 ] || exit $rc ;;
    pmc)
      npmc=$((npmc+1))
      (cd /tmp && export TMPDIR=/tmp && cd "$ROOT" && rm -rf gpurun_out/pmc_$npmc && \
        timeout -s KILL 240 rocprofv3 --pmc $(echo "$val" | tr ',' ' ') -d gpurun_out/pmc_$npmc -o run -- \
        python3 bench.py --steps 2 --warmup 1 --graph 0 > gpurun_out/pmc_$npmc.log 2>&1); rc=$?
      tail -2 gpurun_out/pmc_$npmc.log; [ $rc -eq 0 ] || exit $rc ;;
    py)
      scr=${val%%:*}; a=""; [ "$scr" != "$val" ] && a=${val#*:}
      log=gpurun_out/$(basename "$scr" .py).log
      timeout -k 10 600 python -u $scr $a > "$log" 2>&1; rc=$?
      tail -20 "$log"; [ $rc -eq 0 ] || exit $rc ;;
    dist)
      a=${val:-"--steps 3 --warmup 2 --batch 64"}
      BIGDL_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 $a > gpurun_out/dist.log 2>&1; rc=$?
      tail -3 gpurun_out/dist.log; [ $rc -eq 0 ] || exit $rc ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
