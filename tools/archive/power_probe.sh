set -u
O=gpurun_out/pw1; mkdir -p $O
for d in randn bf16 zeros; do
 for h in 1 0; do
  PU_CONV_HALO=$h timeout -k 10 200 python tools/conv_bench.py --layers top,l2,l3 --ops fwd,dgrad,wgrad --data $d > $O/cb_${d}_$h.txt 2>&1 || { tail -20 $O/cb_${d}_$h.txt; exit 1; }
  echo "== $d halo=$h"; grep -v amdgpu.ids $O/cb_${d}_$h.txt | grep -v peak
 done
done
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_halo_conv_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-200
