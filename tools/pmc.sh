#!/bin/bash
# PMC passes over tools/conv_bench.py (one --pmc group per rocprofv3 run, no sys/runtime trace),
# then tools/pmc_summary.py.
#   bash tools/pmc.sh <layers> [outdir] [ops] [extra conv_bench flags, e.g. --bf16]
set -u
LAYERS=${1:-top}
OUT=${2:-gpurun_out/pmc}
OPS=${3:-fwd,dgrad,wgrad}
EXTRA=${4:-}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/p$i -o run -- \
      python tools/conv_bench.py --layers $LAYERS --ops $OPS --reps 3 $EXTRA > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i [$grp] rc=$rc" >> $OUT/passes.log
  [ $rc -eq 0 ] || exit $rc
done <<'GROUPS'
SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE
SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC
FETCH_SIZE
WRITE_SIZE
GROUPS
python tools/pmc_summary.py $OUT > $OUT/summary.txt 2>&1
