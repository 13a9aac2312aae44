#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) over conv_bench top fwd: round-4 vs ping-pong Winograd
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r05pmc
mkdir -p $OUT
for v in 0 1; do
  i=0
  while read -r grp; do
    [ -z "$grp" ] && continue
    i=$((i+1))
    PU_WINO_PP=$v timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/v$v/p$i -o run -- \
        python tools/conv_bench.py --layers ${1:-top} --ops fwd --reps 3 > $OUT/v$v.p$i.log 2>&1
    rc=$?
    echo "v$v pass $i [$grp] rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done <<'GROUPS'
SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VMEM SQ_INST_LEVEL_VMEM SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY
SQ_IFETCH SQ_IFETCH_LEVEL SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SMEM GRBM_GUI_ACTIVE
SQC_ICACHE_MISSES SQC_DCACHE_MISSES SQ_WAVES SQ_INST_LEVEL_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA
TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum SQ_WAVES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE
GROUPS
  mkdir -p $OUT/v$v
  python tools/pmc_summary.py $OUT/v$v > $OUT/v$v/summary.txt 2>&1
done
grep -A40 "wino" $OUT/v0/summary.txt | head -60
grep -A40 "wino" $OUT/v1/summary.txt | head -60
