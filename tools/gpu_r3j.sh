set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
for g in 3 5 3 5; do
  BIGDL_CONV_G4=$g timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --graph 0 > gpurun_out/bench_g4_$g.log 2>&1 || { tail -20 gpurun_out/bench_g4_$g.log; exit 1; }
  echo "g4=$g $(tail -1 gpurun_out/bench_g4_$g.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"]["final_loss"])')"
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 3 --graph 0 > gpurun_out/prof_bench.log 2>&1; rc=$?
tail -2 gpurun_out/prof_bench.log | cut -c1-300
exit $rc
