#!/bin/bash
set -u
O=gpurun_out/r04m; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "pointwise or wgrad or convT" --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 300 python -u -m pytest tests/test_configs_gpu.py -x -q --timeout 250 --timeout-method thread > $O/t2.log 2>&1 || { tail -40 $O/t2.log; exit 1; }
tail -1 $O/t2.log
for c in c4 c2; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-oja > $O/$c.log 2>&1 || { tail -20 $O/$c.log; exit 1; }
done
python - $O <<'PY'
import json, sys
for f in ("c4.log", "c2.log"):
    d = json.loads(open(sys.argv[1] + "/" + f).read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d.get("build_id"))
    for k, v in list((d.get("kernels") or {}).items())[:10]:
        print("  %-28s %s" % (k, v))
PY
bash tools/r04_t4.sh
