# interleaved A/B of one env switch on the training step: gpu_ab2.sh VAR "v1 v2" rounds
export PYTHONPATH=$PWD
VAR=$1; VALS=$2; R=${3:-2}
for i in $(seq 1 $R); do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/ab2.log 2>&1 || { tail -20 gpurun_out/ab2.log; exit 1; }
    echo "$VAR=$v round $i $(tail -1 gpurun_out/ab2.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
