#!/bin/bash
# bf16 small-grid lean tiles (PU_BF16_SMALLT): parity under each tile, then C3 alternating.
set -u
O=gpurun_out/smallt
mkdir -p $O
for T in 128x64 64x64; do
  PU_BF16_SMALLT=$T timeout -k 10 300 python -u -m pytest tests/test_bf16_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest_$T.log 2>&1 || { tail -30 $O/pytest_$T.log; exit 1; }
  echo "$T: $(tail -1 $O/pytest_$T.log)"
done
for r in 1 2; do
  for T in 128x128 128x64 64x64; do
    PU_BF16_SMALLT=$T timeout -k 10 200 python bench.py --config c3 --no-cpu-baseline --no-oja > $O/c3_${T}_$r.log 2>&1 || { tail -20 $O/c3_${T}_$r.log; exit 1; }
    python -c "
import json; d=json.loads(open('$O/c3_${T}_$r.log').read().strip().splitlines()[-1])
print('$T', $r, d['value'], d['ms_per_step'], ' | '.join('%s %.4f' % (k, v['ms_per_step']) for k, v in d['kernels'].items() if 'lean' in k or 'splitk' in k))"
  done
done
