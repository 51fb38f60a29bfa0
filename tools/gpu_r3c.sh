set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --via-optimizer --steps 20 --warmup 5 > gpurun_out/bench_viaopt.log 2>&1 || { tail -20 gpurun_out/bench_viaopt.log; exit 1; }
tail -1 gpurun_out/bench_viaopt.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_plain.log 2>&1 && tail -1 gpurun_out/bench_plain.log
bash tools/gpu_pmc_layer.sh
