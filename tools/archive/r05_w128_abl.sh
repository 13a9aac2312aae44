#!/bin/bash
# Ablations (timing only) of the 64- and 128-channel Winograd items on l3 / l4 (conv_bench, fwd)
set -u
for lib in default libplastic_unet_w2a1.so libplastic_unet_w2a2.so; do
  for v in 1; do  # 128-channel items opt-in
    if [ $lib = default ]; then E=""; else E="PLASTIC_UNET_LIB=plastic-unet_amd/lib/$lib"; fi
    echo "== $lib PU_WINO128=$v"
    env $E PU_WINO128=$v timeout -k 10 200 python tools/conv_bench.py --layers l2,l3,l4 --ops fwd 2>&1 | grep -v "amdgpu.ids\|peak" || exit 1
  done
done
for lib in default libplastic_unet_w1a2.so libplastic_unet_w1a5.so; do
  if [ $lib = default ]; then E=""; else E="PLASTIC_UNET_LIB=plastic-unet_amd/lib/$lib"; fi
  echo "== $lib PU_WINO128=0"
  env $E PU_WINO128=0 timeout -k 10 200 python tools/conv_bench.py --layers l2,l3,l4 --ops fwd 2>&1 | grep -v "amdgpu.ids\|peak" || exit 1
done
