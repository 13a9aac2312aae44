#!/bin/bash
# A/B of the fp32 3x3 convolutions: direct 6-product kernels (PU_WINO=0) vs Winograd (PU_WINO=1),
# tools/conv_bench.py fwd + dgrad at the C2 layer shapes (bs 32).   bash tools/ab_wino.sh [layers]
set -u
L=${1:-top,top_cat,l2,l2_cat,l3,l4,l4_cat,bottom}
for v in 0 1 0 1; do
  echo "== PU_WINO=$v"
  PU_WINO=$v timeout -k 10 150 python tools/conv_bench.py --layers $L --ops fwd,dgrad 2>&1 | grep -v amdgpu.ids || exit 1
done
