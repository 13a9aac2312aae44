#!/bin/bash
# bf16 batched epilogue: bf16 + config parity suites, then C3 A/B against the variant library.
set -u
O=gpurun_out/epib
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_bf16_gpu.py tests/test_configs_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for lib in default libplastic_unet_bold.so; do
    if [ $lib = default ]; then E=""; else E="PLASTIC_UNET_LIB=plastic-unet_amd/lib/$lib"; fi
    env $E timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --no-oja > $O/c3_${lib}_$rep.log 2>&1 || { tail -20 $O/c3_${lib}_$rep.log; exit 1; }
    tail -1 $O/c3_${lib}_$rep.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); ks=d['kernels']; top=sorted(ks.items(), key=lambda kv:-kv[1]['ms_per_step'])[:6]
print('$lib', d['value'], d['ms_per_step'], ' | '.join('%s %.3f' % (k, v['ms_per_step']) for k, v in top))"
  done
done
