# full -m gpu suite + smoke + the four bench configs (no CPU baseline); one GPU call
set -u
mkdir -p gpurun_out/r06f
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06f/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r06f/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06f/smoke.log 2>&1 || { tail -5 gpurun_out/r06f/smoke.log; exit 1; }
tail -1 gpurun_out/r06f/smoke.log
for c in c2 c3 c4 c5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > gpurun_out/r06f/bench_$c.out 2> gpurun_out/r06f/bench_$c.err || exit 1
  tail -1 gpurun_out/r06f/bench_$c.out > gpurun_out/r06f/bench_$c.json
  python -c "import json;d=json.load(open('gpurun_out/r06f/bench_$c.json'));print('$c', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"
done
