#!/bin/bash
# Scalar (non-packed) fp32 subtractions in the Winograd V formation / wgrad plane split: parity,
# then conv_bench and C2 per library (default = both scalar; wsc0 = Winograd fwd packed; wws0 =
# Winograd wgrad packed).
set -u
O=gpurun_out/scalar
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_wino_gpu.py tests/test_precision_gpu.py tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for lib in default libplastic_unet_wsc0.so libplastic_unet_wws0.so; do
    if [ $lib = default ]; then E=""; else E="PLASTIC_UNET_LIB=plastic-unet_amd/lib/$lib"; fi
    echo "== $lib (rep $r)"
    env $E timeout -k 10 200 python tools/conv_bench.py --layers top,l2,l3,l4 --ops fwd,dgrad,wgrad 2>&1 | grep -v "amdgpu.ids\|peak" || exit 1
    env $E timeout -k 10 200 python bench.py --no-cpu-baseline --no-oja > $O/c2_${lib}_$r.log 2>&1 || { tail -20 $O/c2_${lib}_$r.log; exit 1; }
    echo "c2 $lib: $(tail -1 $O/c2_${lib}_$r.log | cut -c60-120)"
  done
done
