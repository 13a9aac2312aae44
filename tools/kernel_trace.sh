#!/bin/bash
# kernel traces of short bench runs (per (kernel, grid) averages) for the given configs
#   bash tools/kernel_trace.sh <tag> [configs...]
set -u
OUT=gpurun_out/${1:-ktrace}; shift
CFGS=${@:-c2 c3}
mkdir -p $OUT
export TMPDIR=/tmp
for c in $CFGS; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$c -o run -- python bench.py --config $c --steps 5 --warmup 3 --no-cpu-baseline --no-oja --no-kernel-profile > $OUT/bench_$c.log 2>&1 || { tail -5 $OUT/bench_$c.log; exit 1; }
  python tools/trace_table.py $(find $OUT/prof_$c -name '*.db' | head -1) > $OUT/table_$c.txt && head -30 $OUT/table_$c.txt | cut -c1-130
done
