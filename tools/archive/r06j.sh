set -u
# wino4 persistent blocks (next item's loads before the output exchange) vs one item per block
mkdir -p gpurun_out/r06j
timeout -k 10 400 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_wino_gpu.py > gpurun_out/r06j/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r06j/pytest.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for v in 0 1; do
  echo "== PU_W4_PERSIST=$v"
  PU_W4_PERSIST=$v timeout -k 10 150 python tools/conv_bench.py --layers top,top_cat,l2,l3,l4 --ops fwd,dgrad 2>&1 | grep -v amdgpu.ids | grep -v peak || exit 1
done; done
for rep in 1 2; do for v in 0 1; do
  PU_W4_PERSIST=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-oja --no-kernel-profile > gpurun_out/r06j/c2_$v.json 2> gpurun_out/r06j/c2_$v.err || { tail -5 gpurun_out/r06j/c2_$v.err; exit 1; }
  echo -n "C2 PU_W4_PERSIST=$v "; tail -1 gpurun_out/r06j/c2_$v.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
done; done
