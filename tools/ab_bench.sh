#!/bin/bash
# End-to-end A/B of one environment switch on bench.py (C2 unless more args): alternating runs.
#   bash tools/ab_bench.sh VAR "v1 v2" [bench args...]
set -u
VAR=$1; VALS=$2; shift 2
for rep in 1 2; do
  for v in $VALS; do
    log=gpurun_out/ab/$VAR.$(basename $v).log
    mkdir -p gpurun_out/ab; env $VAR=$v timeout -k 10 240 python bench.py --no-cpu-baseline --no-oja "$@" > $log 2>&1 || { echo "bench failed ($VAR=$v)"; tail -20 $log; exit 1; }
    out=$(grep "^{\"metric\"" $log | tail -1)
    python -c "
import json,sys; d=json.loads(sys.argv[1]); r=d['roofline']
print('$VAR=$(basename $v)', d['value'], 'img/s', d['ms_per_step'], 'ms', r['kernel'], r['frac'], r.get('direct_equivalent_frac'))" "$out"
  done
done
