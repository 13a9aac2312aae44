#!/bin/bash
# 32-row fused-head blocks at nbf >= 256: head / kernel parity suites, then C5 / C4 benches
set -u
O=gpurun_out/r04_t10
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_res_gpu.py tests/test_configs_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for c in c5 c4; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $O/$c.log 2>&1 || { tail -20 $O/$c.log; exit 1; }
  echo "$c: $(tail -1 $O/$c.log | cut -c1-120)"
done
python - <<'PY'
import json
for c in ("c5", "c4"):
    d = json.loads(open("gpurun_out/r04_t10/%s.log" % c).read().strip().splitlines()[-1])
    print(c, {k: v for k, v in d["kernels"].items() if "head" in k or "plastic" in k})
    print(c, d["oja_update"])
PY
