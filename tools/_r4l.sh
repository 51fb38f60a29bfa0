export PYTHONPATH=$PWD
for i in 1; do
BIGDL_BENCH_TRACE=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/benchtr_$i.log 2>&1 || { tail -20 gpurun_out/benchtr_$i.log; exit 1; }
grep "gaps\|GiB after" gpurun_out/benchtr_$i.log | cut -c1-900
done
BIGDL_BENCH_TRACE=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --graph 0 > gpurun_out/benchtr_g0.log 2>&1 || exit 1
grep "GiB after" gpurun_out/benchtr_g0.log | cut -c1-900
