# rocprofv3 kernel traces of bench.py (eager) under two settings of one environment knob: prof_ab.sh VAR V0 V1
set -o pipefail
export PYTHONPATH=$PWD
ROOT=$PWD
for v in "$2" "$3"; do
  (cd /tmp && export TMPDIR=/tmp && cd "$ROOT" && rm -rf gpurun_out/prof_$v && \
    export "$1=$v" && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$v -o run -- \
    python3 bench.py --steps 5 --warmup 3 --graph 0 > gpurun_out/prof_$v.log 2>&1) || exit 1
  tail -1 gpurun_out/prof_$v.log | cut -c1-160
done
