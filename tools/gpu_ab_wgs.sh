export PYTHONPATH=$PWD; mkdir -p gpurun_out
for i in 1 2; do
  for cfg in ${WGS_CFGS:-"512 256" "1024 256" "768 256" "1024 512"}; do
    set -- $cfg
    BIGDL_WGRAD_WGS=$1 BIGDL_WGRAD_HALO_WGS=$2 timeout -k 10 240 python bench.py --steps 30 --warmup 10 > gpurun_out/wgs.log 2>&1 || exit 1
    echo "WGS=$1 HALO_WGS=$2 round $i $(python -c "import json;d=json.loads(open('gpurun_out/wgs.log').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['value'])")"
  done
done
