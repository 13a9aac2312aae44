#!/bin/bash
# 128-channel Winograd items: Winograd suite, then conv_bench and C2 A/B over PU_WINO128.
set -u
O=gpurun_out/w128
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_wino_gpu.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for v in 1 0; do
    echo "== PU_WINO128=$v (rep $r)"
    PU_WINO128=$v timeout -k 10 200 python tools/conv_bench.py --layers top,top_cat,l2,l2_cat,l3,l4,l4_cat --ops fwd,dgrad > $O/conv_${v}_$r.txt 2>&1 || { tail -20 $O/conv_${v}_$r.txt; exit 1; }
    grep -v amdgpu.ids $O/conv_${v}_$r.txt | grep -v peak
  done
done
VAR=PU_WINO128 VALUES="1 0" CONFIG=c2 PAT=wino bash tools/ab_env_tags.sh
