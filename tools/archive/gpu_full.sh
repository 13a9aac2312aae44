#!/bin/bash
# Full -m gpu suite + C2 bench + the small-channel A/B on C5.
set -u
mkdir -p gpurun_out/full
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/full/pytest.log 2>&1 || { tail -40 gpurun_out/full/pytest.log; exit 1; }
tail -1 gpurun_out/full/pytest.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/full/c2.log 2>&1 || { tail -20 gpurun_out/full/c2.log; exit 1; }
grep '^{"metric"' gpurun_out/full/c2.log | tail -1 > gpurun_out/full/c2.json
python -c "
import json; d=json.load(open('gpurun_out/full/c2.json')); r=d['roofline']
print('C2', d['value'], d['ms_per_step'], r['kernel'], r['frac'], r.get('direct_equivalent_frac'), d['oja_update']['fused_head_bs32']['hbm_frac'])
for k, v in list(d['kernels'].items())[:14]: print('  %-40s %s' % (k, v))"
timeout -k 10 600 bash tools/ab_bench.sh PU_SMALLX6 "0 1" --config c5
