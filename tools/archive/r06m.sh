set -u
# Winograd weight gradient on one wave per SIMD (PU_WW4=1): bit-identity, fp64 bounds, A/B timing
mkdir -p gpurun_out/r06m
timeout -k 10 400 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_wino_gpu.py -k "wgrad" > gpurun_out/r06m/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r06m/pytest.log
[ $rc -eq 0 ] || exit $rc
PU_WW4=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_wino_gpu.py -k "wgrad_vs_fp64" > gpurun_out/r06m/pytest_ww4.log 2>&1; rc=$?
tail -2 gpurun_out/r06m/pytest_ww4.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for v in 0 1; do
  echo "== PU_WW4=$v"
  PU_WW4=$v timeout -k 10 150 python tools/conv_bench.py --layers top,top_cat,l2,l3,l4 --ops wgrad 2>&1 | grep -v amdgpu.ids | grep -v peak || exit 1
done; done
for rep in 1 2; do for v in 0 1; do
  PU_WW4=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-oja --no-kernel-profile > gpurun_out/r06m/c2_$v.json 2> gpurun_out/r06m/c2_$v.err || { tail -5 gpurun_out/r06m/c2_$v.err; exit 1; }
  echo -n "C2 PU_WW4=$v "; tail -1 gpurun_out/r06m/c2_$v.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
done; done
