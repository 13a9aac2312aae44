#!/bin/bash
# Pipelined fused head + one-launch small-channel wgrad reduction: parity (kernels, variants,
# configs), head_bench, C5 / C4 / C2 bench lines.     bash tools/gpu_r03e.sh
set -u
OUT=gpurun_out/r03e
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_variants_gpu.py tests/test_configs_gpu.py tests/test_model_gpu.py -x -q \
    --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2; do timeout -k 10 120 python tools/head_bench.py head 2>&1 | grep head || exit 1; done
for c in c5 c4 c2; do
  timeout -k 10 240 python bench.py --config $c --no-cpu-baseline > $OUT/$c.log 2>&1 || { tail -20 $OUT/$c.log; exit 1; }
  grep "^{\"metric\"" $OUT/$c.log | tail -1 > $OUT/$c.json
  python -c "
import json; d=json.load(open('$OUT/$c.json')); r=d['roofline']; o=d.get('oja_update',{})
print('$c', d['value'], d['ms_per_step'], r['kernel'], r['frac'], {k: v.get('hbm_frac') for k, v in o.items() if 'fused' in k})"
done
