#!/bin/bash
# A/B of the default library against a variant .so on one bench config, printing the kernel-table
# rows whose tag contains PAT:   TESTS="tests/x.py ..." PAT=x6 CONFIG=c2 bash tools/ab_lib_tags.sh variant.so
set -u
O=gpurun_out/abl
mkdir -p $O
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
for r in 1 2 3; do
  for lib in default $1; do
    if [ $lib = default ]; then E=""; else E="PLASTIC_UNET_LIB=plastic-unet_amd/lib/$lib"; fi
    env $E timeout -k 10 200 python bench.py --config ${CONFIG:-c2} --no-cpu-baseline --no-oja > $O/$lib.$r.log 2>&1 || { tail -20 $O/$lib.$r.log; exit 1; }
    tail -1 $O/$lib.$r.log | python -c "
import json,sys; d=json.loads(sys.stdin.read())
ks=d['kernels']; sel=[(k, v) for k, v in ks.items() if '${PAT:-}' in k]
print('$lib r$r', d['value'], d['ms_per_step'], ' | '.join('%s %.0fx%.3f' % (k, v['launches_per_step'], v['ms_per_step']) for k, v in sel))"
  done
done
