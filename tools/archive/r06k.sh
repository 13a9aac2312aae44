set -u
# wino4 one-round output exchange (default) vs the 3-round exchange (PU_W4_XCH1=0 build)
mkdir -p gpurun_out/r06k
timeout -k 10 400 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_wino_gpu.py > gpurun_out/r06k/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/r06k/pytest.log
[ $rc -eq 0 ] || exit $rc
PLASTIC_UNET_LIB=plastic-unet_amd/lib/libplastic_unet_w4st.so timeout -k 10 200 python tools/w4_items.py top l4 2>&1 | grep -v amdgpu.ids | grep -v xcc || exit 1
for rep in 1 2; do for v in "" x3; do
  echo "== ${v:-release}"
  PLASTIC_UNET_LIB=plastic-unet_amd/lib/libplastic_unet${v:+_$v}.so timeout -k 10 150 python tools/conv_bench.py --layers top,top_cat,l2,l3,l4 --ops fwd,dgrad 2>&1 | grep -v amdgpu.ids | grep -v peak || exit 1
done; done
for rep in 1 2; do for v in "" x3; do
  PLASTIC_UNET_LIB=plastic-unet_amd/lib/libplastic_unet${v:+_$v}.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-oja --no-kernel-profile > gpurun_out/r06k/c2_$v.json 2> gpurun_out/r06k/c2_$v.err || { tail -5 gpurun_out/r06k/c2_$v.err; exit 1; }
  echo -n "C2 ${v:-release} "; tail -1 gpurun_out/r06k/c2_$v.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
done; done
