#!/bin/bash
# Winograd source before the batched epilogue (libplastic_unet_wold.so, f02bccb's winograd.hip) vs
# the current one: conv_bench per layer and C2, alternating on one box.
set -u
O=gpurun_out/wold
mkdir -p $O
for r in 1 2; do
  for lib in default libplastic_unet_wold.so; do
    if [ $lib = default ]; then E=""; else E="PLASTIC_UNET_LIB=plastic-unet_amd/lib/$lib"; fi
    echo "== $lib (rep $r)"
    env $E timeout -k 10 200 python tools/conv_bench.py --layers top,l2,l3,l4 --ops fwd,dgrad 2>&1 | grep -v "amdgpu.ids\|peak" || exit 1
    env $E timeout -k 10 200 python bench.py --no-cpu-baseline --no-oja --no-kernel-profile > $O/c2_${lib}_$r.log 2>&1 || { tail -20 $O/c2_${lib}_$r.log; exit 1; }
    echo "c2 $lib: $(tail -1 $O/c2_${lib}_$r.log | cut -c60-125)"
  done
done
