#!/bin/bash
# kernel traces of short bench runs: per (kernel, grid) average durations; C4/C5 kernel tables
set -u
OUT=gpurun_out/${1:-ktrace}
mkdir -p $OUT
export TMPDIR=/tmp
for c in c2 c3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$c -o run -- python bench.py --config $c --steps 5 --warmup 3 --no-cpu-baseline --no-oja --no-kernel-profile > $OUT/bench_$c.log 2>&1 || { tail -5 $OUT/bench_$c.log; exit 1; }
  python tools/trace_table.py $(find $OUT/prof_$c -name '*kernel_trace.csv' | head -1) > $OUT/table_$c.txt && head -45 $OUT/table_$c.txt
done
for c in c4 c5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-oja > $OUT/$c.log 2>&1 || { tail -20 $OUT/$c.log; exit 1; }
done
python - $OUT <<'PY'
import json, sys
for f in ("c4.log", "c5.log"):
    d = json.loads(open(sys.argv[1] + "/" + f).read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d.get("build_id"))
    for k, v in list((d.get("kernels") or {}).items())[:18]:
        print("  %-28s %s" % (k, v))
PY
