# Fused-head A/B: head_bench.py on the release library and the listed variants (same box, alternating).
#   bash tools/ab_head.sh fh_nt fh_u4 ...   (variants from tools/build_variant.py; HEAD_SHAPE="B N C")
set -u
for round in 1 2; do
  for v in default "$@"; do
    if [ $v = default ]; then lib=plastic-unet_amd/lib/libplastic_unet.so; else lib=plastic-unet_amd/lib/libplastic_unet_$v.so; fi
    PLASTIC_UNET_LIB=$lib timeout -k 10 120 python tools/head_bench.py $v ${HEAD_SHAPE:-} 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
