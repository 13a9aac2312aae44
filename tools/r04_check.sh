#!/bin/bash
# Round-4 GPU check: the -m gpu suite, the C2 bench, per-layer conv timings.  bash tools/r04_check.sh tag
set -u
TAG=${1:-r04}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python bench.py > $O/c2.log 2>&1 || { tail -20 $O/c2.log; exit 1; }
tail -1 $O/c2.log | cut -c1-400
timeout -k 10 200 python tools/conv_bench.py --layers top,top_cat,l2,l2_cat,l3,l4,l4_cat --ops fwd,dgrad,wgrad > $O/conv.txt 2>&1 || { tail -20 $O/conv.txt; exit 1; }
grep -v amdgpu.ids $O/conv.txt
