set -u
mkdir -p gpurun_out/r06d
for v in 0 1 0 1; do
  PU_WINO4=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-oja > gpurun_out/r06d/bench_w$v.out 2>gpurun_out/r06d/bench_w$v.err || exit 1
  tail -1 gpurun_out/r06d/bench_w$v.out > gpurun_out/r06d/bench_w$v.json
  python -c "import json;d=json.load(open('gpurun_out/r06d/bench_w$v.json'));r=d['roofline'];print('PU_WINO4=$v', d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_us'], r['frac'], r['direct_equivalent_frac'])"
done
