#!/bin/bash
# Jupyter notebook server with bigdl_amd on the path (reference jupyter-with-bigdl.sh).
set -euo pipefail
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)"
export PYTHONPATH="$HERE${PYTHONPATH:+:$PYTHONPATH}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
command -v jupyter >/dev/null || { echo "jupyter is not installed in this environment" >&2; exit 1; }
exec jupyter notebook --ip "${JUPYTER_IP:-127.0.0.1}" --port "${JUPYTER_PORT:-8888}" --no-browser "$@"
