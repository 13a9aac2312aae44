# x6 lean igemm MFMA-order timing ablations (abl_order2 computes wrong sums: timing only)
set -u
O=gpurun_out/ablo; mkdir -p $O
for rep in 1 2; do
for v in base order1 order2; do
  if [ $v = base ]; then L=plastic-unet_amd/lib/libplastic_unet.so; else L=plastic-unet_amd/lib/abl_$v.so; fi
  PLASTIC_UNET_LIB=$L timeout -k 10 120 python tools/conv_bench.py --layers top,l2,l3 --ops fwd,dgrad --reps 30 > $O/$v.$rep.log 2>&1 || exit 1
  echo "== $v ($rep)"; grep -v "amdgpu.ids\|peak" $O/$v.$rep.log
done
done
