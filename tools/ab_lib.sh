#!/bin/bash
# A/B of two builds of the library (the default and a variant .so under plastic-unet_amd/lib):
# Winograd tests on the default, then conv_bench + the C2 bench alternating.
#   bash tools/ab_lib.sh tag variant.so [layers] [ops]
set -u
TAG=$1
VAR=plastic-unet_amd/lib/$2
L=${3:-top,top_cat,l2,l3,l4}
OPS=${4:-fwd,dgrad,wgrad}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_wino_gpu.py -x -q --timeout 200 --timeout-method thread > $O/wino.log 2>&1 || { tail -40 $O/wino.log; exit 1; }
tail -1 $O/wino.log
for rep in 1 2; do
  for lib in default $2; do
    echo "== $lib (rep $rep)"
    if [ $lib = default ]; then E=""; else E="PLASTIC_UNET_LIB=$VAR"; fi
    env $E timeout -k 10 200 python tools/conv_bench.py --layers $L --ops $OPS > $O/conv_${lib}_$rep.txt 2>&1 || { tail -20 $O/conv_${lib}_$rep.txt; exit 1; }
    grep -v amdgpu.ids $O/conv_${lib}_$rep.txt
  done
done
for lib in default $2 default $2; do
  if [ $lib = default ]; then E=""; else E="PLASTIC_UNET_LIB=$VAR"; fi
  env $E timeout -k 10 300 python bench.py --no-cpu-baseline --no-oja > $O/c2_$lib.log 2>&1 || { tail -20 $O/c2_$lib.log; exit 1; }
  echo "c2 $lib: $(tail -1 $O/c2_$lib.log | cut -c1-150)"
done
