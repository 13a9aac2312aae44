#!/bin/bash
# Iteration check in one GPU call: the -m gpu suite, then the C2 bench line (+ optional extra args).
#   bash tools/gpu_quick.sh TAG [bench args...]
set -u
TAG=${1:-quick}; shift || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $OUT/c2.log 2>&1 || { tail -20 $OUT/c2.log; exit 1; }
tail -1 $OUT/c2.log > $OUT/c2.json
python -c "
import json; d=json.load(open('$OUT/c2.json'))
print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d['oja_update']['fused_head_bs32'])"
