#!/bin/bash
# round-4 Winograd kernel variants (PU_WINO_PP=0): conv_bench top / top_cat / l2 / l3 fwd + dgrad
set -u
export PU_WINO_PP=0
for t in ${1:-wP wS wPS}; do
  echo "== $t"
  PLASTIC_UNET_LIB=plastic-unet_amd/lib/libplastic_unet_$t.so timeout -k 10 120 python tools/conv_bench.py --layers ${2:-top,top_cat,l2,l3} --ops fwd,dgrad 2>&1 | grep -v "amdgpu.ids\|peak" || exit 1
done
echo "== release"
timeout -k 10 120 python tools/conv_bench.py --layers ${2:-top,top_cat,l2,l3} --ops fwd,dgrad 2>&1 | grep -v "amdgpu.ids\|peak"
