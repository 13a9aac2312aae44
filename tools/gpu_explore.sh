#!/bin/bash
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1; echo "list rc=$?" >> $OUT/explore.log
timeout -k 10 900 python -m pytest tests -m gpu -q -s -p no:cacheprovider --timeout 600 > $OUT/tests.log 2>&1; rc=$?
echo "tests rc=$rc" >> $OUT/explore.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python tools/conv_bench.py --json $OUT/conv_bench.json > $OUT/conv_bench.log 2>&1; rc=$?
echo "conv_bench rc=$rc" >> $OUT/explore.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py --no-cpu-baseline > $OUT/bench.log 2>&1; rc=$?
echo "bench rc=$rc" >> $OUT/explore.log
