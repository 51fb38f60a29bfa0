set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --graph 0 > gpurun_out/bench_eager.log 2>&1; tail -1 gpurun_out/bench_eager.log
