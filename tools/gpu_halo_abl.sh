# halo kernel K-loop ablations (BIGDL_CONV_HALO_ABL: 1 no epilogue, +2 no MFMA, +4 no DMA in the loop, +8 no LDS reads)
export PYTHONPATH=$PWD
for abl in 1 3 5 9 13 15; do
  BIGDL_CONV_HALO_ABL=$abl timeout -k 10 200 python tools/conv_variants.py --layers 2,10,16,22 --ops fwd_nostats --variants "abl$abl:chalo=1" --rounds 3 > gpurun_out/halo_abl_$abl.log 2>&1 || { tail -5 gpurun_out/halo_abl_$abl.log; exit 1; }
  echo "== ABL $abl"; grep -v amdgpu.ids gpurun_out/halo_abl_$abl.log | tail -4
done
