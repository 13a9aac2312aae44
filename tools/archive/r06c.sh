set -u
for v in "" w4s1 w4s2 w4pe; do
  echo "== ${v:-release}"
  if [ -n "$v" ]; then export PLASTIC_UNET_LIB=plastic-unet_amd/lib/libplastic_unet_$v.so; fi
  timeout -k 10 120 python tools/conv_bench.py --layers top,l2,l3,l4 --ops fwd,dgrad 2>&1 | grep -v amdgpu.ids | grep -v peak || exit 1
done
