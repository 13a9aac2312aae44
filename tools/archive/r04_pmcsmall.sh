#!/bin/bash
# PMC of the 8-channel MFMA conv (C5's 512^2 level, bs 16) + its conv_bench timing
set -u
timeout -k 10 120 python tools/conv_bench.py --layers s8,s8_cat,s16 --ops fwd,dgrad --batch 16 2>&1 | grep -v amdgpu.ids || exit 1
bash tools/pmc.sh s8 gpurun_out/r04z fwd,dgrad "--batch 16" || exit 1
grep -A 40 "smallconv_x6_kernel<8, 8>" gpurun_out/r04z/summary.txt | head -42
