#!/bin/bash
# Winograd iteration: parity tests, per-layer A/B, PMC of the top / l3 forward, end-to-end A/B.
set -u
mkdir -p gpurun_out/wino
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -k "wino or precision" > gpurun_out/wino/pytest.log 2>&1 || { tail -30 gpurun_out/wino/pytest.log; exit 1; }
tail -1 gpurun_out/wino/pytest.log
timeout -k 10 400 bash tools/ab_wino.sh top,top_cat,l2,l2_cat,l3,l4 > gpurun_out/wino/ab.txt 2>&1 || { tail -20 gpurun_out/wino/ab.txt; exit 1; }
cat gpurun_out/wino/ab.txt
PU_WINO=1 bash tools/pmc.sh top,l3 gpurun_out/wino/pmc fwd || exit 1
timeout -k 10 600 bash tools/ab_bench.sh PU_WINO "0 1" > gpurun_out/wino/e2e.txt 2>&1; cat gpurun_out/wino/e2e.txt
