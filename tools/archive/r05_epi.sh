#!/bin/bash
# Batched epilogues (igemm x6 / Winograd): kernel parity suites, then A/B against a variant library.
#   bash tools/r05_epi.sh TAG variant.so
set -u
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_wino_gpu.py tests/test_precision_gpu.py tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/ab_lib.sh $1 $2 top,top_cat,l2,l2_cat,l3,l4,l4_cat fwd,dgrad
