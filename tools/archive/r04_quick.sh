#!/bin/bash
# quick GPU validation: Winograd / kernel / model tests, fused head A/B, per-layer wgrad, C2 bench
set -u
TAG=${1:-r04q}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_wino_gpu.py tests/test_kernels_gpu.py tests/test_precision_gpu.py tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
for v in 1 0 1 0; do PU_HEAD_PIPE=$v timeout -k 10 120 python tools/head_bench.py "pipe=$v" 2>&1 | grep -v amdgpu.ids || exit 1; done
timeout -k 10 200 python tools/conv_bench.py --layers top,top_cat,l2,l2_cat,l3,l4,l4_cat,bottom --ops wgrad > $O/conv.txt 2>&1 || { tail -20 $O/conv.txt; exit 1; }
grep -v amdgpu.ids $O/conv.txt
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c2.log 2>&1 || { tail -20 $O/c2.log; exit 1; }
python - $O/c2.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("c2", d["value"], d["ms_per_step"], d.get("build_id"), "fused head", d.get("oja_update", {}).get("fused_head_bs32"))
for k, v in list((d.get("kernels") or {}).items())[:14]:
    print("  %-28s %s" % (k, v))
PY
