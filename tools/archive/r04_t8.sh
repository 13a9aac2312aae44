#!/bin/bash
# ConvT forward on the small-channel MFMA kernel: parity suites, conv timing, then C5 / C4 benches
set -u
O=gpurun_out/r04_t8
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_res_gpu.py tests/test_kernels_gpu.py tests/test_variants_gpu.py tests/test_configs_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python tools/conv_bench.py --layers s8,s8_cat,s16 --ops fwd,dgrad --batch 16 > $O/conv.txt 2>&1 || { tail -20 $O/conv.txt; exit 1; }
grep TF $O/conv.txt
for c in c5 c4 c5 c4; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-oja > $O/$c.log 2>&1 || { tail -20 $O/$c.log; exit 1; }
  echo "$c: $(tail -1 $O/$c.log | cut -c1-120)"
done
python - <<'PY'
import json
for c in ("c5",):
    d = json.loads(open("gpurun_out/r04_t8/%s.log" % c).read().strip().splitlines()[-1])
    for k, v in d["kernels"].items():
        if "x6s" in k or "igemm<256x64,x6>" in k:
            print(c, k, v)
PY
