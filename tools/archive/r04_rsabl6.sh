#!/bin/bash
set -u
for v in default rsabl6 rsabl2; do
  if [ $v = default ]; then L=""; else L="PLASTIC_UNET_LIB=plastic-unet_amd/lib/libplastic_unet_$v.so"; fi
  echo "== $v"
  env $L timeout -k 10 120 python tools/conv_bench.py --bf16 --layers top --ops fwd,dgrad 2>&1 | grep -v amdgpu.ids | head -1 || exit 1
done
