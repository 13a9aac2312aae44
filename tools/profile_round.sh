#!/bin/bash
# Round profile of the default bench: rocprofv3 kernel-trace stats, then separate PMC passes
# (FETCH_SIZE / WRITE_SIZE / clock + MFMA busy - never combined with sys/runtime traces).
#   bash tools/profile_round.sh [tag]      -> gpurun_out/prof/ ; copy summaries into profiles/
set -u
TAG=${1:-r01}
OUT=gpurun_out/prof
mkdir -p $OUT
export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- $B > $OUT/bench_stats.log 2>&1 || exit $?
echo "stats ok" >> $OUT/passes.log
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -o run -- $B --steps 3 --warmup 1 > $OUT/fetch.log 2>&1 || exit $?
echo "fetch ok" >> $OUT/passes.log
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -o run -- $B --steps 3 --warmup 1 > $OUT/write.log 2>&1 || exit $?
echo "write ok" >> $OUT/passes.log
timeout -k 10 600 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace --output-format csv -d $OUT/clock -o run -- $B --steps 3 --warmup 1 > $OUT/clock.log 2>&1 || exit $?
echo "clock ok" >> $OUT/passes.log
python tools/pmc_traffic.py $OUT $OUT/pmc_traffic.json > $OUT/pmc_traffic.txt 2>&1
