#!/bin/bash
# Launch a bigdl_amd program on the GPUs of this node, one process per GPU over RCCL / xGMI.
# MI355X counterpart of the reference's spark-submit-with-bigdl.sh: torch.distributed.run replaces
# spark-submit, ranks replace executors.
#
#   scripts/run-with-bigdl.sh [-n NGPU] [--nnodes N --node-rank R --master HOST:PORT] [--dry-run] prog.py [args]
set -euo pipefail
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)"
NGPU=""
NNODES=1
NODE_RANK=0
MASTER="127.0.0.1:29500"
DRY=0
while [ $# -gt 0 ]; do
  case "$1" in
    -n|--nproc-per-node) NGPU="$2"; shift 2 ;;
    --nnodes) NNODES="$2"; shift 2 ;;
    --node-rank) NODE_RANK="$2"; shift 2 ;;
    --master) MASTER="$2"; shift 2 ;;
    --dry-run) DRY=1; shift ;;
    -h|--help) sed -n 2,7p "$0"; exit 0 ;;
    *) break ;;
  esac
done
[ $# -ge 1 ] || { echo "usage: $0 [-n NGPU] prog.py [args]" >&2; exit 2; }
if [ -z "$NGPU" ]; then
  NGPU=$(python3 -c "import torch; print(max(1, torch.cuda.device_count()))" 2>/dev/null || echo 1)
fi
export PYTHONPATH="$HERE${PYTHONPATH:+:$PYTHONPATH}"
export HSA_ENABLE_IPC_MODE_LEGACY=0          # dmabuf IPC: RCCL / cross-process tensor sharing
export OMP_NUM_THREADS="${OMP_NUM_THREADS:-8}"
CMD=(python3 -m torch.distributed.run --nnodes "$NNODES" --node-rank "$NODE_RANK" --nproc-per-node "$NGPU"
     --master-addr "${MASTER%:*}" --master-port "${MASTER##*:}" "$@")
if [ "$DRY" = 1 ]; then echo "${CMD[*]}"; exit 0; fi
exec "${CMD[@]}"
