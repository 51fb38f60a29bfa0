set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
run() {  # name, env...
  name=$1; shift
  env "$@" BIGDL_BENCH_TRACE=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --graph 0 > gpurun_out/bench_$name.log 2>&1 || { tail -20 gpurun_out/bench_$name.log; exit 1; }
  echo "$name $(tail -1 gpurun_out/bench_$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])') $(grep 'host enqueue' gpurun_out/bench_$name.log)"
}
echo "OMP_NUM_THREADS=$OMP_NUM_THREADS"
run h_default
run h_omp1 OMP_NUM_THREADS=1
run h_spin0 GOMP_SPINCOUNT=0
run h_default2
