#!/bin/bash
# High-priority data-gradient stream (PU_HIPRIO) A/B on C3: bitwise side-stream tests under it, then
# C3 alternating.
set -u
O=gpurun_out/hiprio
mkdir -p $O
PU_HIPRIO=1 timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -k side_stream -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
python -c "import torch; print('priority range', torch.cuda.Stream.priority_range())"
for r in 1 2 3; do
  for H in 0 1; do
    PU_HIPRIO=$H timeout -k 10 200 python bench.py --config c3 --no-cpu-baseline --no-oja --no-kernel-profile > $O/c3_${H}_$r.log 2>&1 || { tail -20 $O/c3_${H}_$r.log; exit 1; }
    python -c "
import json; d=json.loads(open('$O/c3_${H}_$r.log').read().strip().splitlines()[-1]); print('hiprio $H rep $r', d['value'], d['ms_per_step'])"
  done
done
