#!/bin/bash
# Round-4 GPU check: Winograd tests (wino2 4-wave default + 8-wave variant), the -m gpu suite,
# C2 benches per Winograd kernel, per-layer conv timings.   bash tools/r04_check.sh tag [full]
set -u
TAG=${1:-r04}
FULL=${2:-full}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_wino_gpu.py -x -q --timeout 200 --timeout-method thread > $O/wino.log 2>&1 || { tail -40 $O/wino.log; exit 1; }
tail -2 $O/wino.log
PU_WINO_KERNEL=3 timeout -k 10 400 python -u -m pytest tests/test_wino_gpu.py -x -q --timeout 200 --timeout-method thread -k "fwd_dgrad or persistent" > $O/wino3.log 2>&1 || { tail -40 $O/wino3.log; exit 1; }
tail -2 $O/wino3.log
for k in 1 2 3; do
  echo "== PU_WINO_KERNEL=$k"
  PU_WINO_KERNEL=$k timeout -k 10 200 python tools/conv_bench.py --layers top,top_cat,l2,l2_cat,l3,l4,bottom --ops fwd,dgrad > $O/conv_k$k.txt 2>&1 || { tail -20 $O/conv_k$k.txt; exit 1; }
  grep -v amdgpu.ids $O/conv_k$k.txt
done
for v in 1 0; do
  echo "== PU_WINO_WGRAD=$v"
  PU_WINO_WGRAD=$v timeout -k 10 200 python tools/conv_bench.py --layers top,top_cat,l2,l2_cat,l3,l4,l4_cat,bottom --ops wgrad > $O/conv_wg$v.txt 2>&1 || { tail -20 $O/conv_wg$v.txt; exit 1; }
  grep -v amdgpu.ids $O/conv_wg$v.txt
done
for k in 2 3 1; do
  PU_WINO_KERNEL=$k timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c2_k$k.log 2>&1 || { tail -20 $O/c2_k$k.log; exit 1; }
  echo "c2 kernel $k: $(tail -1 $O/c2_k$k.log | cut -c1-200)"
done
if [ "$FULL" = full ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
