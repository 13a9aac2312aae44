set -u
for v in default abl1; do
  if [ $v = default ]; then lib=plastic-unet_amd/lib/libplastic_unet.so; else lib=plastic-unet_amd/lib/libpu_fh_$v.so; fi
  PLASTIC_UNET_LIB=$lib timeout -k 10 120 python tools/head_bench.py $v 2>&1 | grep -v amdgpu.ids || exit 1
done
