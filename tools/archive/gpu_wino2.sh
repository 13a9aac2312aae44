#!/bin/bash
set -u
mkdir -p gpurun_out/wino
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -k "wino" > gpurun_out/wino/pytest.log 2>&1 || { tail -30 gpurun_out/wino/pytest.log; exit 1; }
tail -1 gpurun_out/wino/pytest.log
for v in 0 1 0 1; do echo "== PU_WINO_PERSIST=$v"; PU_WINO_PERSIST=$v timeout -k 10 100 python tools/conv_bench.py --layers top,top_cat,l2,l3,l4 --ops fwd,dgrad 2>&1 | grep -v amdgpu.ids || exit 1; done
PU_WINO_PERSIST=0 bash tools/pmc.sh top gpurun_out/wino/pmc_top fwd || exit 1
PU_WINO_PERSIST=0 bash tools/pmc.sh l3 gpurun_out/wino/pmc_l3 fwd || exit 1
python tools/pmc_summary.py gpurun_out/wino/pmc_top | sed -n '/wino_x6/,$p'
python tools/pmc_summary.py gpurun_out/wino/pmc_l3 | sed -n '/wino_x6/,$p'
