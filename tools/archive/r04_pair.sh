#!/bin/bash
# row-pair small-channel conv: parity tests, then conv_bench + C5/C4 A/B against PU_SX_PAIR=0
set -u
O=gpurun_out/r04_pair
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_variants_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for lib in default nopair; do
    if [ $lib = default ]; then E=""; else E="PLASTIC_UNET_LIB=plastic-unet_amd/lib/libplastic_unet_nopair.so"; fi
    env $E timeout -k 10 200 python tools/conv_bench.py --layers s8,s8_cat --ops fwd,dgrad --batch 16 > $O/conv_${lib}_$rep.txt 2>&1 || { tail -20 $O/conv_${lib}_$rep.txt; exit 1; }
    echo "== $lib (rep $rep)"; grep TF $O/conv_${lib}_$rep.txt
  done
done
for c in c5 c4; do
  for lib in default nopair default nopair; do
    if [ $lib = default ]; then E=""; else E="PLASTIC_UNET_LIB=plastic-unet_amd/lib/libplastic_unet_nopair.so"; fi
    env $E timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-oja > $O/${c}_$lib.log 2>&1 || { tail -20 $O/${c}_$lib.log; exit 1; }
    echo "$c $lib: $(tail -1 $O/${c}_$lib.log | cut -c1-130)"
  done
done
