set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/diag_graph_fusion.py > gpurun_out/diag_graph_fusion.log 2>&1; rc=$?
cat gpurun_out/diag_graph_fusion.log | tail -130
exit $rc
