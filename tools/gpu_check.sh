#!/bin/bash
# GPU-box session: tests, smoke, bench, rocprofv3 summary.  Stops at the first crash/timeout
# (exit codes other than 0/1), never retries a GPU step.
set -u
OUT=gpurun_out
mkdir -p $OUT
step() {  # name, timeout, command...
    local name=$1; local tmo=$2; shift 2
    echo "== $name" >> $OUT/session.log
    timeout -k 10 $tmo "$@" > $OUT/$name.log 2>&1
    local rc=$?
    echo "== $name exit=$rc" >> $OUT/session.log
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)" >> $OUT/session.log; exit $rc; fi
    return 0
}
MODE=${1:-all}
if [ "$MODE" = "all" ] || [ "$MODE" = "tests" ]; then
  step tests 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$MODE" = "all" ] || [ "$MODE" = "bench" ]; then
  step bench 900 python bench.py ${BENCH_ARGS:-}
fi
if [ "$MODE" = "all" ] || [ "$MODE" = "prof" ]; then
  export TMPDIR=/tmp
  step rocprof 900 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
fi
tail -3 $OUT/session.log
