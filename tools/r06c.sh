set -u
export PU_WINO4=1
for v in "" w4a1 w4a2 w4a4 w4a5; do
  echo "== ${v:-release}"
  if [ -n "$v" ]; then export PLASTIC_UNET_LIB=plastic-unet_amd/lib/libplastic_unet_$v.so; fi
  timeout -k 10 120 python tools/conv_bench.py --layers top,l3,l4 --ops fwd 2>&1 | grep -v amdgpu.ids | grep -v peak || exit 1
done
