#!/bin/bash
# LDS / texture-path PMC passes over tools/conv_bench.py (one --pmc group per run, no traces):
#   bash tools/pmc_lds.sh <layers> <outdir> <ops>   -> <outdir>/summary.txt
set -u
LAYERS=${1:-top}
OUT=${2:-gpurun_out/pmc_lds}
OPS=${3:-fwd}
mkdir -p $OUT
export TMPDIR=/tmp
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/p$i -o run -- \
      python tools/conv_bench.py --layers $LAYERS --ops $OPS --reps 3 > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i [$grp] rc=$rc" >> $OUT/passes.log
  [ $rc -eq 0 ] || exit $rc
done <<'GROUPS'
SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_DATA_FIFO_FULL SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
TA_TA_BUSY_sum TA_BUFFER_TOTAL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum GRBM_GUI_ACTIVE SQ_WAVES
GROUPS
python tools/pmc_summary.py $OUT > $OUT/summary.txt 2>&1
