export PYTHONPATH=$PWD
for cfg in DIAG_TAG=default DIAG_TAG=nowgrad,BIGDL_WGRAD_STREAM=0 DIAG_TAG=inflight1,BIGDL_MAX_INFLIGHT=1 DIAG_TAG=serial,AMD_SERIALIZE_KERNEL=3; do
  IFS=',' read -ra envs <<< "$cfg"
  env "${envs[@]}" timeout -k 10 200 python -u tools/diag_determinism.py 5 2>&1 | grep "rel vs" || exit 1
done
