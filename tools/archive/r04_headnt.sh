#!/bin/bash
set -u
for rep in 1 2 3; do
  timeout -k 10 120 python tools/head_bench.py "default" 2>&1 | grep -v amdgpu.ids || exit 1
  PLASTIC_UNET_LIB=plastic-unet_amd/lib/libplastic_unet_hnt.so timeout -k 10 120 python tools/head_bench.py "nontemporal" 2>&1 | grep -v amdgpu.ids || exit 1
done
