#!/bin/bash
# Round-4 GPU call: -m gpu suite, C2 bench (kernel table), L1 probe, PMC of the Winograd kernels.
#   bash tools/r04_prof.sh tag
set -u
TAG=${1:-r04c}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python bench.py > $O/c2.log 2>&1 || { tail -20 $O/c2.log; exit 1; }
tail -1 $O/c2.log > $O/c2.json
python - $O/c2.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("c2", d["value"], d["ms_per_step"], d.get("build_id"), "roofline", d.get("roofline"))
for k, v in list((d.get("kernels") or {}).items())[:30]:
    print("  %-28s %s" % (k, v))
PY
if [ -x tools/probes/l1_bw ]; then timeout -k 10 60 tools/probes/l1_bw > $O/l1_bw.txt 2>&1; cat $O/l1_bw.txt; fi
bash tools/pmc.sh top,l3 $O/pmc fwd,wgrad || exit 1
bash tools/pmc_lds.sh top,l3 $O/pmc_lds fwd,wgrad || exit 1
grep -A40 "wino_x6_kernel\|wgrad_wino" $O/pmc/summary.txt | head -120
grep -A30 "wino_x6_kernel\|wgrad_wino" $O/pmc_lds/summary.txt | head -80
