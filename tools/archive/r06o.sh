set -u
# wino4: bias + first-row masks loaded before the output exchange (EPI_EARLY) and U one sub-stage
# ahead (UA1); variant libraries: ua42141 = early, ua42041 = early + U one ahead
mkdir -p gpurun_out/r06o
for v in ua42141 ua42041; do
  PLASTIC_UNET_LIB=plastic-unet_amd/lib/libplastic_unet_$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_wino_gpu.py > gpurun_out/r06o/pytest_$v.log 2>&1; rc=$?
  echo -n "$v: "; tail -1 gpurun_out/r06o/pytest_$v.log
  [ $rc -eq 0 ] || exit $rc
done
for rep in 1 2; do for v in "" ua42141 ua42041; do
  echo "== ${v:-release}"
  PLASTIC_UNET_LIB=plastic-unet_amd/lib/libplastic_unet${v:+_$v}.so timeout -k 10 150 python tools/conv_bench.py --layers top,top_cat,l2,l3,l4 --ops fwd,dgrad 2>&1 | grep -v amdgpu.ids | grep -v peak || exit 1
done; done
for rep in 1 2; do for v in "" ua42141 ua42041; do
  PLASTIC_UNET_LIB=plastic-unet_amd/lib/libplastic_unet${v:+_$v}.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-oja --no-kernel-profile > gpurun_out/r06o/c2_$v.json 2> gpurun_out/r06o/c2_$v.err || { tail -5 gpurun_out/r06o/c2_$v.err; exit 1; }
  echo -n "C2 ${v:-release} "; tail -1 gpurun_out/r06o/c2_$v.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
done; done
