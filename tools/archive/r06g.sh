set -u
# 32 x 288 nine-wave wgrad tile (C4/C5 32-channel layers): parity then C5 / C4 bench A/B
mkdir -p gpurun_out/r06g
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_res_gpu.py tests/test_configs_gpu.py > gpurun_out/r06g/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r06g/pytest.log
[ $rc -eq 0 ] || exit $rc
run() {
  local tag=$1; shift
  echo -n "$tag "
  timeout -k 10 300 env "$@" > gpurun_out/r06g/$tag.json 2> gpurun_out/r06g/$tag.err || { echo FAIL; tail -5 gpurun_out/r06g/$tag.err; return 1; }
  tail -1 gpurun_out/r06g/$tag.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
}
for rep in 1 2; do
  for cfg in c5 c4; do
    run ${cfg}_288_$rep PU_WG288=1 python bench.py --config $cfg --steps 20 --warmup 4 --no-cpu-baseline --no-kernel-profile --no-oja || exit 1
    run ${cfg}_128_$rep PU_WG288=0 python bench.py --config $cfg --steps 20 --warmup 4 --no-cpu-baseline --no-kernel-profile --no-oja || exit 1
  done
done
