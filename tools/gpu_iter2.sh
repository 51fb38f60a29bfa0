export PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest tests/test_deterministic_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t6.log 2>&1; rc=$?; tail -5 gpurun_out/t6.log
timeout -k 10 600 python -u tools/det_check.py --iters 10 --r50 > gpurun_out/det.log 2>&1; rc2=$?; cat gpurun_out/det.log | grep -v amdgpu.ids
[ $rc2 -eq 0 ] || exit $rc2
bash tools/gpu_prof_step.sh
