set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.log 2>&1 || { tail -20 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log | cut -c1-1000
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --via-optimizer > gpurun_out/bench_opt.log 2>&1 || { tail -20 gpurun_out/bench_opt.log; exit 1; }
tail -1 gpurun_out/bench_opt.log | cut -c1-1000
