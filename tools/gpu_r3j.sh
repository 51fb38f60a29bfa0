set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
for g in 3 5 3 5; do
  BIGDL_CONV_G4=$g timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --graph 0 > gpurun_out/bench_g4_$g.log 2>&1 || { tail -20 gpurun_out/bench_g4_$g.log; exit 1; }
  echo "g4=$g $(tail -1 gpurun_out/bench_g4_$g.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"]["final_loss"])')"
done
