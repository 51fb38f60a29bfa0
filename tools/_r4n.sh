export PYTHONPATH=$PWD
for v in 0 1; do
BIGDL_BN_BWD_REF=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bnref_$v.log 2>&1 || { tail -20 gpurun_out/bnref_$v.log; exit 1; }
echo "ref=$v $(tail -1 gpurun_out/bnref_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"]["final_loss"])')"
grep -c "not the BN output" gpurun_out/bnref_$v.log; grep "not the BN output" gpurun_out/bnref_$v.log | sort | uniq -c | head -5
done
