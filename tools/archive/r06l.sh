set -u
# fused head: 16 streamer waves x 4 pixels in flight (hs16) vs 8 x 8 (release); bitwise checks first
mkdir -p gpurun_out/r06l
PLASTIC_UNET_LIB=plastic-unet_amd/lib/libplastic_unet_hs16.so timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "head" > gpurun_out/r06l/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/r06l/pytest.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do for v in "" hs16; do
  echo -n "${v:-release} "
  PLASTIC_UNET_LIB=plastic-unet_amd/lib/libplastic_unet${v:+_$v}.so timeout -k 10 120 python tools/head_bench.py 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
done; done
