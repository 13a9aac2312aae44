#!/bin/bash
# fp32 C2 with only the non-Winograd weight gradients (ConvT, stem) on the side stream
# (PU_WSTREAM=light) vs none: side-stream bitwise tests, then C2 alternating.
set -u
O=gpurun_out/light
mkdir -p $O
PU_WSTREAM=light timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -k side_stream -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  for S in 0 light; do
    PU_WSTREAM=$S timeout -k 10 200 python bench.py --no-cpu-baseline --no-oja --no-kernel-profile > $O/c2_${S}_$r.log 2>&1 || { tail -20 $O/c2_${S}_$r.log; exit 1; }
    python -c "
import json; d=json.loads(open('$O/c2_${S}_$r.log').read().strip().splitlines()[-1]); print('wstream $S rep $r', d['value'], d['ms_per_step'])"
  done
done
