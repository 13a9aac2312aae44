set -u
# VA=3 variant: parity (whole Winograd GPU file, variant library) then fwd timing A/B
mkdir -p gpurun_out/r06e
PLASTIC_UNET_LIB=plastic-unet_amd/lib/libplastic_unet_w4va3.so timeout -k 10 400 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_wino_gpu.py > gpurun_out/r06e/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r06e/pytest.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
bash tools/r06c.sh || exit 1
done
