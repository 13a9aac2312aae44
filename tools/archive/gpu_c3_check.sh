#!/bin/bash
# bf16 (config C3) iteration: the bf16 parity tests, conv A/B (halo vs per-tap lean), the C3 bench.
set -u
O=gpurun_out/${1:-c3}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_bf16_gpu.py tests/test_configs_gpu.py -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for h in 1 0; do
  PU_CONV_HALO=$h timeout -k 10 200 python tools/conv_bench.py --bf16 --layers top,top_cat,l2,l2_cat,l3 --ops fwd,dgrad > $O/cb_$h.txt 2>&1 || { tail -20 $O/cb_$h.txt; exit 1; }
  echo "== halo=$h"; grep -v amdgpu.ids $O/cb_$h.txt
done
timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline > $O/bench_c3.log 2>&1 || { tail -20 $O/bench_c3.log; exit 1; }
tail -1 $O/bench_c3.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step']); [print(k, v) for k,v in list(d['kernels'].items())[:10]]"
