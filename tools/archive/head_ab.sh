#!/bin/bash
# fused head variants: pipelined 8+4 waves (default library), phase-serial (PU_HEAD_PIPE=0), 12+4 lib
set -u
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q -k "head or fused or model" --timeout 200 --timeout-method thread 2>&1 | tail -1 || exit 1
PLASTIC_UNET_LIB=plastic-unet_amd/lib/libplastic_unet_hp12.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "head or fused" --timeout 200 --timeout-method thread 2>&1 | tail -1 || exit 1
for rep in 1 2; do
  timeout -k 10 120 python tools/head_bench.py "pipe 8+4" 2>&1 | grep -v amdgpu.ids || exit 1
  PU_HEAD_PIPE=0 timeout -k 10 120 python tools/head_bench.py "serial" 2>&1 | grep -v amdgpu.ids || exit 1
  PLASTIC_UNET_LIB=plastic-unet_amd/lib/libplastic_unet_hp12.so timeout -k 10 120 python tools/head_bench.py "pipe rot" 2>&1 | grep -v amdgpu.ids || exit 1
done
bash tools/r04_next.sh r04n
