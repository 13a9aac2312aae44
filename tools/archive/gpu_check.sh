#!/bin/bash
# One GPU call: the -m gpu parity suite, the default C2 bench line, then the rocprofv3 kernel-trace
# stats of the same bench (a separate run: profiled runs clock lower).  Each step has its own time
# limit and the chain stops at the first failure.
#   bash tools/gpu_check.sh [tag] [--no-tests]
set -u
TAG=${1:-r02}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
if [ "${2:-}" != "--no-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
  tail -3 $OUT/pytest.log
fi
timeout -k 10 300 python bench.py > $OUT/bench_c2.log 2>&1 || { tail -30 $OUT/bench_c2.log; exit 1; }
tail -1 $OUT/bench_c2.log | cut -c 1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python bench.py --no-cpu-baseline --no-oja > $OUT/bench_rocprof.log 2>&1 || { tail -30 $OUT/bench_rocprof.log; exit 1; }
echo done
