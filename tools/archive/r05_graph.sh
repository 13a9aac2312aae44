#!/bin/bash
# HIP-graph training step: bitwise test vs eager, then bench C3 / C4 / C2 with and without graphs.
set -u
O=gpurun_out/graph
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -k graph_step -x -q --timeout 250 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for c in c3 c4 c2; do
  for G in graph eager; do
    if [ $G = eager ]; then E="--graph off"; else E="--graph on"; fi
    timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-oja $E > $O/${c}_$G.log 2>&1 || { tail -30 $O/${c}_$G.log; exit 1; }
    python -c "
import json; d=json.loads(open('$O/${c}_$G.log').read().strip().splitlines()[-1]); print('$c $G', d['value'], d['ms_per_step'], d['config'].get('step_launch'), d['final_loss'])"
  done
done
