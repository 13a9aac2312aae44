#!/bin/bash
# Round profile of the FINAL build, one GPU call:
#   1. the C2 bench line (bench.py defaults)                          -> $OUT/c2.json
#   2. rocprofv3 --kernel-trace --stats of the same command             -> $OUT/c2_stats/
#   3. separate PMC passes (FETCH_SIZE / WRITE_SIZE / clock + MFMA busy; never combined with
#      sys/runtime traces) and tools/pmc_traffic.py                      -> $OUT/pmc_traffic.json
#   4. C3 bench line + its kernel-trace stats, C4 and C5 bench lines     -> $OUT/c{3,4,5}.json
# Every step has its own time limit; the chain stops at the first failure.
#   bash tools/profile_round.sh [tag]   (then copy the summaries into profiles/)
set -u
TAG=${1:-r02}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
B="python bench.py"
step() { echo "[$(date +%T)] $1" | tee -a $OUT/passes.log; }

step "c2 bench"
timeout -k 10 300 $B > $OUT/c2.log 2>&1 || { tail -20 $OUT/c2.log; exit 1; }
tail -1 $OUT/c2.log > $OUT/c2.json
step "c2 kernel-trace stats"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c2_stats -o run -- \
    $B --no-cpu-baseline --no-oja > $OUT/c2_stats.log 2>&1 || { tail -20 $OUT/c2_stats.log; exit 1; }
grep "^{\"metric\"" $OUT/c2_stats.log | tail -1 > $OUT/c2_under_rocprof.json
for pass in "fetch FETCH_SIZE" "write WRITE_SIZE" "clock GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES"; do
  set -- $pass
  name=$1; shift
  step "pmc $name ($*)"
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $OUT/$name -o run -- \
      $B --no-cpu-baseline --no-oja --no-kernel-profile --steps 3 --warmup 1 > $OUT/$name.log 2>&1 \
      || { tail -20 $OUT/$name.log; exit 1; }
done
python tools/pmc_traffic.py $OUT $OUT/pmc_traffic.json > $OUT/pmc_traffic.txt 2>&1 || { cat $OUT/pmc_traffic.txt; exit 1; }
step "c3 bench"
timeout -k 10 300 $B --config c3 > $OUT/c3.log 2>&1 || { tail -20 $OUT/c3.log; exit 1; }
tail -1 $OUT/c3.log > $OUT/c3.json
step "c3 kernel-trace stats"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c3_stats -o run -- \
    $B --config c3 --no-cpu-baseline --no-oja > $OUT/c3_stats.log 2>&1 || { tail -20 $OUT/c3_stats.log; exit 1; }
for pass in "fetch FETCH_SIZE" "write WRITE_SIZE" "clock GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES"; do
  set -- $pass
  name=$1; shift
  step "c3 pmc $name ($*)"
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $OUT/c3pmc/$name -o run -- \
      $B --config c3 --no-cpu-baseline --no-oja --no-kernel-profile --steps 3 --warmup 1 > $OUT/c3pmc_$name.log 2>&1 \
      || { tail -20 $OUT/c3pmc_$name.log; exit 1; }
done
python tools/pmc_traffic.py $OUT/c3pmc $OUT/c3_pmc_traffic.json > $OUT/c3_pmc_traffic.txt 2>&1 || { cat $OUT/c3_pmc_traffic.txt; exit 1; }
step "c4 bench"
timeout -k 10 300 $B --config c4 > $OUT/c4.log 2>&1 || { tail -20 $OUT/c4.log; exit 1; }
tail -1 $OUT/c4.log > $OUT/c4.json
step "c5 bench"
timeout -k 10 300 $B --config c5 > $OUT/c5.log 2>&1 || { tail -20 $OUT/c5.log; exit 1; }
tail -1 $OUT/c5.log > $OUT/c5.json
step "done"
