#!/bin/bash
# Lazy direct operands: model / DP parity, then C2 A/B over PU_LAZY_DIRECT.
set -u
mkdir -p gpurun_out/lazy
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py tests/test_dp_gpu.py tests/test_res_gpu.py tests/test_coord_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/lazy/pytest.log 2>&1 || { tail -40 gpurun_out/lazy/pytest.log; exit 1; }
tail -1 gpurun_out/lazy/pytest.log
VAR=PU_LAZY_DIRECT VALUES="1 0" CONFIG=c2 bash tools/ab_env_bench.sh
