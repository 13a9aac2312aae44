#!/bin/bash
# Clock and MFMA-busy of the x6 lean igemm on random vs zero operands (the power-limit evidence of
# DESIGN.md section 2): one PMC pass per data mode, counters GRBM_GUI_ACTIVE + SQ_VALU_MFMA_BUSY_CYCLES.
set -u
OUT=${1:-gpurun_out/pmc_power}
mkdir -p $OUT
export TMPDIR=/tmp
for d in randn zeros; do
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES --kernel-trace --output-format csv -d $OUT/$d/p1 -o run -- \
      python tools/conv_bench.py --layers top,l2,l3 --ops fwd --reps 5 --data $d > $OUT/$d.log 2>&1 || exit $?
  python tools/pmc_summary.py $OUT/$d > $OUT/summary_$d.txt 2>&1 || exit $?
done
