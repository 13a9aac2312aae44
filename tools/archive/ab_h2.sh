set -u
for v in 2 1; do
  echo "== PU_CONV_HALO=$v"
  PU_CONV_HALO=$v timeout -k 10 120 python tools/conv_bench.py --bf16 --layers top,top_cat,l2,l3 --ops fwd,dgrad 2>&1 | grep -v amdgpu.ids | head -4 || exit 1
done
