set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof_g1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_g1 -o run -- python3 bench.py --steps 5 --warmup 3 --graph 1 > gpurun_out/prof_g1.log 2>&1; rc=$?
tail -1 gpurun_out/prof_g1.log | cut -c1-200
exit $rc
