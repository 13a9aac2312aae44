#!/bin/bash
# Round-final suite + profile of the product build, then the C = 16 small-channel conv on an 8-row
# tile (lib/libplastic_unet_sx8.so, PU_SX16_TH=8 variant) vs the product: parity, per-layer timing,
# C5 A/B.     bash tools/gpu_r03i.sh
set -u
bash tools/round_final.sh r03i || exit 1
OUT=gpurun_out/r03i
L=$PWD/plastic-unet_amd/lib
PLASTIC_UNET_LIB=$L/libplastic_unet_sx8.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "small" -x -q --timeout 150 --timeout-method thread > $OUT/pytest_sx8.log 2>&1 || { tail -30 $OUT/pytest_sx8.log; exit 1; }
tail -1 $OUT/pytest_sx8.log
for v in "" _sx8; do
  PLASTIC_UNET_LIB=$L/libplastic_unet$v.so timeout -k 10 120 python tools/conv_bench.py --batch 16 --layers s8_cat,s16,s16_cat --ops fwd,dgrad 2>&1 | grep -v amdgpu.ids || exit 1
done
bash tools/ab_bench.sh PLASTIC_UNET_LIB "$L/libplastic_unet.so $L/libplastic_unet_sx8.so" --config c5 || exit 1
