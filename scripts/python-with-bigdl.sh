#!/bin/bash
# Python (or an interactive shell) with bigdl_amd importable and the engine environment set
# (reference pyspark-with-bigdl.sh). Extra arguments go to python3.
set -euo pipefail
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)"
export PYTHONPATH="$HERE${PYTHONPATH:+:$PYTHONPATH}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
exec python3 "$@"
