# Full GPU tier + smoke + 1-GPU bench, each step under its own time limit (run from the repo root via gpurun).
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/gpu_tier.log 2>&1 &&
tail -3 gpurun_out/gpu_tier.log &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 &&
tail -1 gpurun_out/smoke.log &&
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err &&
tail -1 gpurun_out/bench.log
