set -o pipefail
O=gpurun_out/r2s52
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d $O/p1 -o run --output-format csv -- python3 bench.py --topology fabric100k-w --steps 1 --warmup 0 --iso-reps 0 --no-cpu > $O/p1.log 2>&1 || { echo P1_FAIL; tail -5 $O/p1.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/p2 -o run --output-format csv -- python3 bench.py --topology fabric100k-w --steps 1 --warmup 0 --iso-reps 0 --no-cpu > $O/p2.log 2>&1 || { echo P2_FAIL; tail -5 $O/p2.log; exit 1; }
python3 scripts/pmc_by_kernel.py $O/p1 $O/p2 > $O/pmc.json
python3 - <<PY
import json
d=json.load(open('$O/pmc.json'))
for k,v in d.items():
    wc=v.get('SQ_WAVE_CYCLES',0)
    if not wc or 'wderive' not in k and 'cover' not in k: continue
    print(k, v['dispatches'], {c: round(v.get(c,0)/wc,3) for c in ('SQ_WAIT_ANY','SQ_WAIT_INST_ANY','SQ_ACTIVE_INST_ANY','SQ_ACTIVE_INST_VALU','SQ_ACTIVE_INST_LDS')}, 'lds_instr', v.get('SQ_INSTS_LDS',0)/1e6, 'bankconf', v.get('SQ_LDS_BANK_CONFLICT',0)/1e6, 'valu', v.get('SQ_INSTS_VALU',0)/1e9, 'vmrd', v.get('SQ_INSTS_VMEM_RD',0)/1e6, 'salu', v.get('SQ_INSTS_SALU',0)/1e9, 'waves', v.get('SQ_WAVES',0), 'busy', v.get('SQ_BUSY_CYCLES',0)/1e6, 'gui', v.get('GRBM_GUI_ACTIVE',0)/1e6)
PY
