#!/bin/bash
# Build the gfx950 kernels in-tree and package a wheel under dist/ (reference make-dist.sh / python_package.sh).
set -euo pipefail
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)"
cd "$HERE"
export PYTORCH_ROCM_ARCH=gfx950
python3 setup.py build_ext --inplace
python3 setup.py bdist_wheel -d dist
ls -l dist
