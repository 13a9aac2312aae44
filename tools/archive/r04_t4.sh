#!/bin/bash
set -u
O=gpurun_out/r04o; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_bf16_gpu.py tests/test_res_gpu.py -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
PU_BF16_LEAN128=1 timeout -k 10 300 python -u -m pytest tests/test_bf16_gpu.py -x -q --timeout 200 --timeout-method thread > $O/t128.log 2>&1 || { tail -40 $O/t128.log; exit 1; }
tail -1 $O/t128.log
for v in 1 0; do
  PU_BF16_ROWS=$v timeout -k 10 200 python tools/conv_bench.py --bf16 --layers top --ops fwd,dgrad > $O/convbf_$v.txt 2>&1 || { tail -20 $O/convbf_$v.txt; exit 1; }
  echo "== PU_BF16_ROWS=$v"; grep -v amdgpu.ids $O/convbf_$v.txt
done
PU_BF16_LEAN128=1 timeout -k 10 200 python tools/conv_bench.py --bf16 --layers l4,bottom --ops fwd,dgrad > $O/convbf_l128.txt 2>&1 || { tail -20 $O/convbf_l128.txt; exit 1; }
timeout -k 10 200 python tools/conv_bench.py --bf16 --layers l4,bottom --ops fwd,dgrad > $O/convbf_l256.txt 2>&1 || { tail -20 $O/convbf_l256.txt; exit 1; }
echo "== lean 128 / default"; grep -v amdgpu.ids $O/convbf_l128.txt $O/convbf_l256.txt
for v in rows norows lean128; do
  case $v in rows) E="";; norows) E="PU_BF16_ROWS=0";; lean128) E="PU_BF16_LEAN128=1";; esac
  env $E timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --no-oja > $O/c3_$v.log 2>&1 || { tail -20 $O/c3_$v.log; exit 1; }
done
python - $O <<'PY'
import json, sys
for f in ("c3_rows.log", "c3_norows.log", "c3_lean128.log"):
    d = json.loads(open(sys.argv[1] + "/" + f).read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d.get("build_id"))
    for k, v in list((d.get("kernels") or {}).items())[:8]:
        print("  %-28s %s" % (k, v))
PY
