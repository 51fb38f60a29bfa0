export PYTHONPATH=$PWD
for v in 1 0; do
  BIGDL_CONV_P8=$v timeout -k 10 400 python -u tools/conv_roofline.py --iters 10 > gpurun_out/roofline_p8_$v.txt 2>&1 || exit 1
  tail -5 gpurun_out/roofline_p8_$v.txt
done
bash tools/gpu_ab.sh BIGDL_CONV_P8 "1 0" 2
