#!/bin/bash
# bf16 16^2 layers (128 x 128 lean tiles, 256 blocks): K split 2 (PU_BF16_L128SPLIT=1) vs none.
set -u
O=gpurun_out/l128s
mkdir -p $O
PU_BF16_L128SPLIT=1 timeout -k 10 300 python -u -m pytest tests/test_bf16_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  for S in 0 1; do
    PU_BF16_L128SPLIT=$S timeout -k 10 200 python bench.py --config c3 --no-cpu-baseline --no-oja > $O/c3_${S}_$r.log 2>&1 || { tail -20 $O/c3_${S}_$r.log; exit 1; }
    python -c "
import json; d=json.loads(open('$O/c3_${S}_$r.log').read().strip().splitlines()[-1])
print('split $S rep $r', d['value'], d['ms_per_step'], ' | '.join('%s %d x %.4f' % (k, v['launches_per_step'], v['ms_per_step']) for k, v in d['kernels'].items() if 'lean' in k))"
  done
done
