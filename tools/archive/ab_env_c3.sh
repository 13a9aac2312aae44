#!/bin/bash
# C3 bench A/B over one environment variable: bash tools/ab_env_c3.sh VAR "v1 v2 ..." (empty string = unset)
set -u
VAR=$1; VALS=$2
for rep in 1 2; do
  for v in $VALS; do
    if [ "$v" = "-" ]; then E=""; else E="$VAR=$v"; fi
    echo "== $VAR=$v (rep $rep)"
    env $E timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --no-oja 2>&1 | tail -1 | python -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d.get('kernels',{})
print(d['value'], d['ms_per_step'], {t: k[t]['ms_per_step'] for t in k if 'wgrad' in t})" || exit 1
  done
done
