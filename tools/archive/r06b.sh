set -u
mkdir -p gpurun_out/r06b
timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_wino_gpu.py -k "wino4" > gpurun_out/r06b/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r06b/pytest.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for v in "PU_WINO4=0" "PU_WINO4=1"; do
  echo "== $v"
  env $v timeout -k 10 150 python tools/conv_bench.py --layers top,top_cat,l2,l2_cat,l3,l4,bottom --ops fwd,dgrad 2>&1 | grep -v amdgpu.ids | grep -v peak || exit 1
done; done
