#!/bin/bash
# Round-4 GPU check: Winograd tests first, the -m gpu suite, the C2 bench, per-layer conv timings
# (weight gradients with the Winograd-domain kernel on / off).   bash tools/r04_check.sh tag [full]
set -u
TAG=${1:-r04}
FULL=${2:-full}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_wino_gpu.py -x -q --timeout 200 --timeout-method thread > $O/wino.log 2>&1 || { tail -40 $O/wino.log; exit 1; }
tail -2 $O/wino.log
if [ "$FULL" = full ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
timeout -k 10 300 python bench.py > $O/c2.log 2>&1 || { tail -20 $O/c2.log; exit 1; }
tail -1 $O/c2.log | cut -c1-300
for v in 1 0; do
  echo "== PU_WINO_WGRAD=$v"
  PU_WINO_WGRAD=$v timeout -k 10 200 python tools/conv_bench.py --layers top,top_cat,l2,l2_cat,l3,l4,l4_cat,bottom --ops wgrad > $O/conv_wg$v.txt 2>&1 || { tail -20 $O/conv_wg$v.txt; exit 1; }
  grep -v amdgpu.ids $O/conv_wg$v.txt
done
