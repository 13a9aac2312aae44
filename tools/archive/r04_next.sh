#!/bin/bash
# wgrad reduction change + bf16 halo A/B (register-staged vs DMA ring) on C3
set -u
TAG=${1:-r04n}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_wino_gpu.py tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_bf16_gpu.py -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-oja > $O/c2.log 2>&1 || { tail -20 $O/c2.log; exit 1; }
for h in 1 2; do
  PU_CONV_HALO=$h timeout -k 10 200 python tools/conv_bench.py --bf16 --layers top,top_cat,l2,l2_cat,l3,l4 --ops fwd,dgrad > $O/convbf_$h.txt 2>&1 || { tail -20 $O/convbf_$h.txt; exit 1; }
  echo "== PU_CONV_HALO=$h"; grep -v amdgpu.ids $O/convbf_$h.txt
  PU_CONV_HALO=$h timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --no-oja > $O/c3_$h.log 2>&1 || { tail -20 $O/c3_$h.log; exit 1; }
done
python - $O <<'PY'
import json, sys
for f in ("c2.log", "c3_1.log", "c3_2.log"):
    d = json.loads(open(sys.argv[1] + "/" + f).read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d.get("build_id"))
    for k, v in list((d.get("kernels") or {}).items())[:12]:
        print("  %-28s %s" % (k, v))
PY
