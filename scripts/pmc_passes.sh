#!/bin/bash
# PMC passes over one command (one rocprofv3 --pmc run per pass, counters
# within the gfx950 per-block slot limits). Usage:
#   bash scripts/pmc_passes.sh <outdir> <command...>
set -u
OUT=$1; shift
export TMPDIR=/tmp
mkdir -p "$OUT"
i=0
for P in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VALU" \
         "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCC_HIT_sum TCC_MISS_sum" \
         "GRBM_GUI_ACTIVE TCC_EA0_RDREQ_sum TCC_REQ_sum TD_TD_BUSY_sum TD_TC_STALL_sum SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P -d "$OUT/p$i" -o run --output-format csv -- "$@" > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
