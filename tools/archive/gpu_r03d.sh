#!/bin/bash
# Fused head: 16 rows per block (product) vs 8 (PU_FH_R=8, 512 blocks at bs 32) - parity of the
# variant on the head tests, then tools/head_bench.py alternating.     bash tools/gpu_r03d.sh
set -u
OUT=gpurun_out/r03d
mkdir -p $OUT
L=$PWD/plastic-unet_amd/lib
PLASTIC_UNET_LIB=$L/libplastic_unet_fhr8.so timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -k "head" -x -q \
    --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2; do
  for v in "" _fhr8; do
    PLASTIC_UNET_LIB=$L/libplastic_unet$v.so timeout -k 10 120 python tools/head_bench.py "head$v" 2>&1 | grep head || exit 1
  done
done
