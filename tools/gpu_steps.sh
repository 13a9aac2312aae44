#!/bin/bash
# Run GPU steps in order; each: NAME TIMEOUT COMMAND... separated by ';;'.  A step's exit status 0/1
# continues, anything else (fault, abort, timeout) stops the session.  Logs: gpurun_out/<NAME>.log
#   bash tools/gpu_steps.sh conv 300 python tools/conv_bench.py ';;' tests 600 python -m pytest ...
set -u
OUT=gpurun_out
mkdir -p $OUT
args=("$@")
i=0
while [ $i -lt ${#args[@]} ]; do
    name=${args[$i]}; tmo=${args[$((i+1))]}; i=$((i+2))
    cmd=()
    while [ $i -lt ${#args[@]} ] && [ "${args[$i]}" != ";;" ]; do cmd+=("${args[$i]}"); i=$((i+1)); done
    i=$((i+1))
    echo "== $name: ${cmd[*]}" >> $OUT/session.log
    timeout -k 10 $tmo "${cmd[@]}" > $OUT/$name.log 2>&1
    rc=$?
    echo "== $name exit=$rc" >> $OUT/session.log
    tail -3 $OUT/$name.log
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
done
