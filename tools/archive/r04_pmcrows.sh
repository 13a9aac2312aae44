#!/bin/bash
# PMC of the bf16 top-level conv: row-stream kernel (default) and the halo kernel (PU_BF16_ROWS=0)
set -u
bash tools/pmc.sh top gpurun_out/r04s/rows fwd --bf16 || exit 1
PU_BF16_ROWS=0 bash tools/pmc.sh top gpurun_out/r04s/halo fwd --bf16 || exit 1
grep -A 40 "rows_kernel" gpurun_out/r04s/rows/summary.txt | head -45
