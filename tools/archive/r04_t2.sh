#!/bin/bash
set -u
O=gpurun_out/r04l; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_wino_gpu.py tests/test_entry_gpu.py tests/test_bf16_gpu.py -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
bash tools/c2_trace.sh r04l c4 c5 c2
