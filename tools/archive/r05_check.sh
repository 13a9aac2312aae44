#!/bin/bash
# Round-5 check: the -m gpu suite, smoke(), then the default C2 bench line (as the driver runs it).
#   bash tools/r05_check.sh TAG
set -u
TAG=${1:-r05}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { tail -40 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || { tail -20 gpurun_out/$TAG/smoke.log; exit 1; }
tail -1 gpurun_out/$TAG/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/$TAG/c2.log 2>&1 || { tail -20 gpurun_out/$TAG/c2.log; exit 1; }
grep '^{"metric"' gpurun_out/$TAG/c2.log | tail -1 > gpurun_out/$TAG/c2.json
python -c "
import json; d=json.load(open('gpurun_out/$TAG/c2.json')); r=d['roofline']
print('C2', d['value'], d['ms_per_step'], r['kernel'], r['frac'], r.get('direct_equivalent_frac'), d['oja_update']['fused_head_bs32'])
print('cpu', d['cpu_baseline']['value'], d['cpu_baseline']['batched']['value'], d['allreduce'])
for k, v in list(d['kernels'].items())[:16]: print('  %-40s %s' % (k, v))"
timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline > gpurun_out/$TAG/c3.log 2>&1 || { tail -20 gpurun_out/$TAG/c3.log; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/$TAG/c3.log').read().strip().splitlines()[-1]); r=d['roofline']
print('C3', d['value'], d['ms_per_step'], r['kernel'], r['frac'])"
timeout -k 10 200 python tools/sustained.py --steps 800 --out gpurun_out/$TAG/sustained_c2.json > gpurun_out/$TAG/sustained.log 2>&1 || { tail -20 gpurun_out/$TAG/sustained.log; exit 1; }
tail -1 gpurun_out/$TAG/sustained.log
