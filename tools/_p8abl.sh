export PYTHONPATH=$PWD
for cfg in BIGDL_P8_ABL=0 BIGDL_P8_ABL=8 BIGDL_P8_ABL=10 BIGDL_P8_ABL=16 BIGDL_P8_ABL=32; do
  echo "== $cfg"; env $cfg timeout -k 10 120 python -u tools/gemm_ceiling.py 2>&1 | grep TF | head -4 || exit 1
done
