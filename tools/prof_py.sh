#!/bin/bash
# rocprofv3 kernel-trace + stats of one python script: tools/prof_py.sh NAME SCRIPT [ARGS...] -> gpurun_out/prof_NAME/
# followed by a per-kernel summary (tools/rocpd_summary.py) in gpurun_out/prof_NAME.txt
set -o pipefail
name=$1; shift
ROOT=$PWD
export PYTHONPATH=$ROOT
cd /tmp && export TMPDIR=/tmp && cd "$ROOT" || exit 1
rm -rf gpurun_out/prof_$name
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$name -o run -- python3 "$@" \
  > gpurun_out/prof_$name.log 2>&1 || { tail -5 gpurun_out/prof_$name.log; exit 1; }
db=$(ls gpurun_out/prof_$name/*.db 2>/dev/null | head -1)
[ -n "$db" ] || db=$(find gpurun_out/prof_$name -name '*.db' | head -1)
python3 tools/rocpd_summary.py kernels "$db" > gpurun_out/prof_$name.txt 2>&1
tail -1 gpurun_out/prof_$name.log; head -12 gpurun_out/prof_$name.txt
