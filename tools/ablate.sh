#!/bin/bash
# Ablation timings (variant libraries built with parts of a kernel removed - timing only, their
# results are wrong): conv_bench per variant next to the default build.
#   bash tools/ablate.sh tag
set -u
TAG=${1:-abl}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_wino_gpu.py -x -q --timeout 200 --timeout-method thread > $O/wino.log 2>&1 || { tail -40 $O/wino.log; exit 1; }
tail -1 $O/wino.log
run() {  # lib label ops
  if [ $1 = default ]; then E=""; else E="PLASTIC_UNET_LIB=plastic-unet_amd/lib/$1"; fi
  env $E timeout -k 10 150 python tools/conv_bench.py --layers top,l3 --ops $2 > $O/$1_$2.txt 2>&1 || { tail -20 $O/$1_$2.txt; exit 1; }
  echo "== $1 ($2)"; grep -E "^(top|l3) " $O/$1_$2.txt
}
for rep in 1 2; do
  run default fwd || exit 1
  for a in 1 2 3 4 5; do run libplastic_unet_wfabl$a.so fwd || exit 1; done
  run default wgrad || exit 1
  for a in 1 2 3 4; do run libplastic_unet_wwabl$a.so wgrad || exit 1; done
done
