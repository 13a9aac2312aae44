#!/bin/bash
# Time the top/l3 conv layers with ablated igemm variants (built in-tree beforehand).
set -u
OUT=gpurun_out; mkdir -p $OUT
for v in 0 1 2 3 4; do
  lib=plastic-unet_amd/lib/libplastic_unet_ablate$v.so
  [ -f $lib ] || continue
  PLASTIC_UNET_LIB=$lib timeout -k 10 300 python tools/conv_bench.py --layers top,l3,bottom --reps 10 > $OUT/ablate$v.log 2>&1
  echo "variant $v rc=$?" >> $OUT/ablate.log
done
