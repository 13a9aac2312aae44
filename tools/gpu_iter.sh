#!/bin/bash
# quick iteration: gpu tests -> conv_bench -> (optional) bench
set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -x > $OUT/tests.log 2>&1; rc=$?
echo "tests rc=$rc" >> $OUT/iter.log; tail -2 $OUT/tests.log >> $OUT/iter.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python tools/conv_bench.py --json $OUT/conv_bench.json > $OUT/conv_bench.log 2>&1; rc=$?
echo "conv_bench rc=$rc" >> $OUT/iter.log
[ $rc -eq 0 ] || exit $rc
if [ "${1:-}" = "bench" ]; then
  timeout -k 10 900 python bench.py --no-cpu-baseline > $OUT/bench.log 2>&1; rc=$?
  echo "bench rc=$rc" >> $OUT/iter.log
fi
