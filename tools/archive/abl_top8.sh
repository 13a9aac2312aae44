# 64-channel lean x6 tile: 4 waves (4x1, 2 pixel fragments per wave) vs 8 waves (8x1, 1 fragment)
set -u
O=gpurun_out/top8; mkdir -p $O
for rep in 1 2; do for v in base top8; do
  if [ $v = base ]; then L=plastic-unet_amd/lib/libplastic_unet.so; else L=plastic-unet_amd/lib/abl_$v.so; fi
  PLASTIC_UNET_LIB=$L timeout -k 10 120 python tools/conv_bench.py --layers top,top_cat --ops fwd,dgrad --reps 30 > $O/$v.$rep.log 2>&1 || exit 1
  echo "== $v ($rep)"; grep -v "amdgpu.ids\|peak" $O/$v.$rep.log
done; done
PLASTIC_UNET_LIB=plastic-unet_amd/lib/abl_top8.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k conv3x3 --timeout 150 --timeout-method thread > $O/pytest.log 2>&1; tail -1 $O/pytest.log
