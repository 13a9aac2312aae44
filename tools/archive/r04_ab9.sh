#!/bin/bash
# A/B: current library vs the previous commit's (lib/libplastic_unet_prev.so): conv_bench small layers, C5 / C4
set -u
O=gpurun_out/r04_ab9
mkdir -p $O
for rep in 1 2; do
  for lib in default prev; do
    if [ $lib = default ]; then E=""; else E="PLASTIC_UNET_LIB=plastic-unet_amd/lib/libplastic_unet_prev.so"; fi
    env $E timeout -k 10 200 python tools/conv_bench.py --layers s8,s8_cat,s16 --ops fwd,dgrad --batch 16 > $O/conv_${lib}_$rep.txt 2>&1 || { tail -20 $O/conv_${lib}_$rep.txt; exit 1; }
    echo "== $lib (rep $rep)"; grep TF $O/conv_${lib}_$rep.txt | cut -c1-110
  done
done
for c in c5 c4; do
  for lib in default prev default prev; do
    if [ $lib = default ]; then E=""; else E="PLASTIC_UNET_LIB=plastic-unet_amd/lib/libplastic_unet_prev.so"; fi
    env $E timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-oja > $O/${c}_$lib.log 2>&1 || { tail -20 $O/${c}_$lib.log; exit 1; }
    echo "$c $lib: $(tail -1 $O/${c}_$lib.log | cut -c1-110)"
  done
done
