#!/bin/bash
# One iteration call: a pytest subset (-k expr), then any number of benchmark commands, each under
# its own time limit; stops at the first failure.   bash tools/gpu_iter.sh TAG 'pytest -k expr' 'cmd1' 'cmd2' ...
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
K=$1; shift
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -k "$K" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
  tail -1 $OUT/pytest.log
fi
i=0
for c in "$@"; do
  i=$((i+1))
  echo "[$(date +%T)] $c"
  timeout -k 10 400 $c > $OUT/cmd$i.log 2>&1 || { tail -30 $OUT/cmd$i.log; exit 1; }
  tail -25 $OUT/cmd$i.log
done
