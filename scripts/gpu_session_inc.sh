# Incremental bench under repair pop budgets (OSPF_REPAIR_POPS).
set -o pipefail
T=${TAG:-s38}
mkdir -p gpurun_out/$T
for P in 8192 2048 512; do
  OSPF_REPAIR_POPS=$P timeout -k 10 600 python -u scripts/bench_incremental.py > gpurun_out/$T/inc_$P.jsonl 2> gpurun_out/$T/inc_$P.err || { echo INC_FAIL; tail -20 gpurun_out/$T/inc_$P.err; exit 1; }
  echo "pops=$P"; python3 -c "
import json
for l in open('gpurun_out/$T/inc_$P.jsonl'):
    d=json.loads(l); print(d['scenario'][:28], d['rerun_roots'], d['repair_ms'], d['rerun_ms'], d['incremental_ms'], d['full_recompute_ms'], d['identical_to_full_rerun'])"
done
