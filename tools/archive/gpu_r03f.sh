#!/bin/bash
# C4/C5 small- and 32-channel layers: per-layer timing and PMC passes (bs 16, as C5).
#   bash tools/gpu_r03f.sh
set -u
OUT=gpurun_out/r03f
mkdir -p $OUT
timeout -k 10 120 python tools/conv_bench.py --batch 16 --layers s8,s8_cat,s16,s16_cat,c32,c32_cat > $OUT/conv.txt 2>&1 || { tail -20 $OUT/conv.txt; exit 1; }
grep -v amdgpu.ids $OUT/conv.txt
bash tools/pmc.sh s8,c32 $OUT/pmc fwd,dgrad,wgrad "--batch 16" || exit 1
grep -E "smallconv|wgrad_small|igemm_x6|wgrad_dma|lean" $OUT/pmc/summary.txt | head -40
