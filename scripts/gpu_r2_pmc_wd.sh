# PMC passes over the weighted rack-switch class (variant 7), one pass per run.
set -o pipefail
T=${TAG:-r2s9}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
CMD="python3 scripts/exp_wdial.py --topology fabric100k-w --roots 8192 --caps 8 --reps 0"
i=0
for P in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_VALU" \
         "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum" \
         "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum" \
         "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum GRBM_GUI_ACTIVE" \
         "SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_VMEM SQ_BUSY_CYCLES GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d $O/p$i -o run --output-format csv -- $CMD > $O/p$i.log 2>&1 || { echo PMC_FAIL $i; tail -5 $O/p$i.log; exit 1; }
  echo pass $i ok
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- $CMD > $O/kt.log 2>&1 || { echo KT_FAIL; tail -5 $O/kt.log; exit 1; }
echo kt ok
