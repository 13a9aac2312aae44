#!/bin/bash
# Round-end bench lines: C2 (default, with the CPU baseline), then C3 / C4 / C5.
set -u
OUT=gpurun_out/final; mkdir -p $OUT
timeout -k 10 900 python bench.py > $OUT/c2.log 2>&1 || exit $?
for c in c3 c4 c5; do
  timeout -k 10 600 python bench.py --config $c --no-cpu-baseline > $OUT/$c.log 2>&1 || exit $?
done
