#!/bin/bash
# Round-3 A/B call: small-channel tests, fused-head phase ablations (tools/head_bench.py over the
# PU_FH_ABL libraries), the small-channel wgrad (row-of-taps items + packed FMA vs
# PU_SW_ROW=0 vs the round-2 form PU_SW_PK=0) and the small-channel MFMA
# conv default (PU_SMALLX6) on C5 / C4.     bash tools/gpu_r03c.sh
set -u
OUT=gpurun_out/r03c
mkdir -p $OUT
L=$PWD/plastic-unet_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_variants_gpu.py tests/test_configs_gpu.py -x -q \
    --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for v in "" _fh1 _fh3 _fh4; do
  PLASTIC_UNET_LIB=$L/libplastic_unet$v.so timeout -k 10 120 python tools/head_bench.py "head$v" >> $OUT/head.txt 2>&1 \
      || { tail -20 $OUT/head.txt; exit 1; }
done
cat $OUT/head.txt
for c in c5 c4; do
  bash tools/ab_bench.sh PLASTIC_UNET_LIB "$L/libplastic_unet.so $L/libplastic_unet_swrow0.so $L/libplastic_unet_swpk0.so" --config $c || exit 1
  bash tools/ab_bench.sh PU_SMALLX6 "0 1" --config $c || exit 1
done
timeout -k 10 120 python tools/diag_fwd.py > $OUT/fwd.txt 2>&1 || { tail -20 $OUT/fwd.txt; exit 1; }
grep flips $OUT/fwd.txt | grep -v "flips 0$" || true
