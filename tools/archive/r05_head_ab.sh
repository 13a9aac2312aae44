#!/bin/bash
# fused-head variants A/B (tools/head_bench.py, bs 32 x 128^2, C = 64), alternating
set -u
for rep in 1 2 3; do
  for t in ${1:-release hNT hU12 hNTU12}; do
    if [ $t = release ]; then unset PLASTIC_UNET_LIB; else export PLASTIC_UNET_LIB=plastic-unet_amd/lib/libplastic_unet_$t.so; fi
    timeout -k 10 60 python tools/head_bench.py $t 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
