#!/bin/bash
# A/B of the fp32 3x3 convolutions, tools/conv_bench.py fwd + dgrad at the C2 layer shapes (bs 32):
# direct 6-product kernels (PU_WINO=0), Winograd one block per item (PU_WINO_PERSIST=0), Winograd
# persistent (default).   bash tools/ab_wino.sh [layers]
set -u
L=${1:-top,top_cat,l2,l2_cat,l3,l4,l4_cat,bottom}
for rep in 1 2; do
  for v in "PU_WINO=0" "PU_WINO=1 PU_WINO_PERSIST=0" "PU_WINO=1"; do
    echo "== $v"
    env $v timeout -k 10 150 python tools/conv_bench.py --layers $L --ops fwd,dgrad 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
