export PYTHONPATH=$PWD
for cfg in BIGDL_CONV_G4=3 BIGDL_CONV_G4=0 BIGDL_CONV_IMPL=2 BIGDL_CONV_W8=2 BIGDL_CONV_G4=7; do
  env $cfg timeout -k 10 120 python -u tools/gemm_ceiling.py 2>&1 | grep TF || exit 1
done
