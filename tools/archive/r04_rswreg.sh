#!/bin/bash
set -u
timeout -k 10 300 python -u -m pytest tests/test_bf16_gpu.py -x -q --timeout 200 --timeout-method thread 2>&1 | tail -1
for v in default rswl default rswl; do
  if [ $v = default ]; then L=""; else L="PLASTIC_UNET_LIB=plastic-unet_amd/lib/libplastic_unet_$v.so"; fi
  echo "== $v"
  env $L timeout -k 10 120 python tools/conv_bench.py --bf16 --layers top --ops fwd,dgrad 2>&1 | grep -v amdgpu.ids | head -1 || exit 1
done
timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --no-oja 2>&1 | tail -1 | cut -c1-150
