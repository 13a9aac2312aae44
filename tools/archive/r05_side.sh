#!/bin/bash
# Side-stream weight gradients (PU_WSTREAM): parity tests, then C2 / C3 A/B.
set -u
mkdir -p gpurun_out/side
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread \
  "tests/test_model_gpu.py::test_c2_side_stream_weight_gradients_bitwise" \
  "tests/test_dp_gpu.py::test_rccl_async_bucket_path_world1" > gpurun_out/side/pytest.log 2>&1 || { tail -40 gpurun_out/side/pytest.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/side/pytest.log
VAR=PU_WSTREAM VALUES="0 1" CONFIG=c2 bash tools/ab_env_bench.sh || exit 1
VAR=PU_WSTREAM VALUES="0 1" CONFIG=c3 bash tools/ab_env_bench.sh || exit 1
