#!/bin/bash
# smallconv register budget: parity of the small-channel kernels, per-layer timing and C5/C4 A/B
# against the previous library (lib/libplastic_unet_prev.so).     bash tools/gpu_r03g.sh
set -u
OUT=gpurun_out/r03g
mkdir -p $OUT
L=$PWD/plastic-unet_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_configs_gpu.py tests/test_variants_gpu.py -x -q \
    --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for v in "" _prev; do
  PLASTIC_UNET_LIB=$L/libplastic_unet$v.so timeout -k 10 120 python tools/conv_bench.py --batch 16 --layers s8,s8_cat,s16,s16_cat --ops fwd,dgrad 2>&1 | grep -v amdgpu.ids || exit 1
done
for c in c5 c4; do
  bash tools/ab_bench.sh PLASTIC_UNET_LIB "$L/libplastic_unet.so $L/libplastic_unet_prev.so" --config $c || exit 1
done
