#!/bin/bash
# pool-level Dropout2d fused into the maxpool kernels: res tests, then two C5 benches
set -u
O=gpurun_out/r04_t6
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_res_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --no-oja > $O/c5_$r.log 2>&1 || { tail -20 $O/c5_$r.log; exit 1; }
  echo "c5: $(tail -1 $O/c5_$r.log | cut -c1-120)"
done
