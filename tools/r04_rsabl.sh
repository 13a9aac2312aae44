#!/bin/bash
# row-stream bf16 conv: fragment prefetch depth A/B (default 4 k-steps, 2, 3) + no-MFMA ablation
set -u
for v in default rspd2 rspd3 rsabl2 default; do
  if [ $v = default ]; then L=""; else L="PLASTIC_UNET_LIB=plastic-unet_amd/lib/libplastic_unet_$v.so"; fi
  echo "== $v"
  env $L timeout -k 10 120 python tools/conv_bench.py --bf16 --layers top --ops fwd,dgrad 2>&1 | grep -v amdgpu.ids | head -1 || exit 1
done
timeout -k 10 300 python -u -m pytest tests/test_bf16_gpu.py -x -q -k rows --timeout 200 --timeout-method thread 2>&1 | tail -1
