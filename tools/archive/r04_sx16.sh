#!/bin/bash
# 16-channel MFMA conv: 8-row tiles (default) vs 16-row (PU_SX16_TH=16 library); C4 / C5 benches
set -u
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_configs_gpu.py tests/test_res_gpu.py -x -q --timeout 250 --timeout-method thread 2>&1 | tail -1
for v in default sx16 default sx16; do
  if [ $v = default ]; then L=""; else L="PLASTIC_UNET_LIB=plastic-unet_amd/lib/libplastic_unet_$v.so"; fi
  echo "== $v"
  env $L timeout -k 10 120 python tools/conv_bench.py --layers s8_cat,s16,s16_cat --ops fwd,dgrad --batch 16 2>&1 | grep -v amdgpu.ids | head -3 || exit 1
done
for c in c5 c4; do
  for v in default sx16; do
    if [ $v = default ]; then L=""; else L="PLASTIC_UNET_LIB=plastic-unet_amd/lib/libplastic_unet_$v.so"; fi
    echo "== $c $v"
    env $L timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-oja 2>&1 | tail -1 | cut -c1-120 || exit 1
  done
done
