set -o pipefail
O=gpurun_out/r2s44
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 bench.py --topology fabric100k-w --mode batch --class-only 96 --reps 1 > $O/kt.log 2>&1 || { echo KT_FAIL; tail -5 $O/kt.log; exit 1; }
bash scripts/pmc_passes.sh $O/pmc python3 bench.py --topology fabric100k-w --mode batch --class-only 96 --reps 1 || { echo PMC_FAIL; exit 1; }
python3 scripts/pmc_by_kernel.py $O/pmc/p1 $O/pmc/p2 $O/pmc/p3 > $O/pmc_by_kernel.json
python3 - <<PY
import csv,glob,json
rows=list(csv.DictReader(open(glob.glob('$O/kt/**/*kernel_stats.csv',recursive=True)[0])))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:6]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.2f} ms {int(r['Calls']):5d} {r['Name'][:70]}")
d=json.load(open('$O/pmc_by_kernel.json'))
for k,v in d.items():
    wc=v.get('SQ_WAVE_CYCLES',0)
    if not wc: continue
    print(k, {c: round(v[c]/wc,3) for c in ('SQ_WAIT_ANY','SQ_WAIT_INST_ANY','SQ_ACTIVE_INST_ANY','SQ_ACTIVE_INST_VALU','SQ_ACTIVE_INST_VMEM')}, 'valu', v['SQ_INSTS_VALU']/1e9, 'vmrd', v['SQ_INSTS_VMEM_RD']/1e6, 'vmwr', v.get('SQ_INSTS_VMEM_WR',0)/1e6, 'lds', v.get('SQ_INSTS_LDS',0)/1e6, 'waves', v.get('SQ_WAVES',0), 'hit', v.get('TCC_HIT_sum',0)/max(1,v.get('TCC_HIT_sum',0)+v.get('TCC_MISS_sum',0)), 'rdreq', v.get('TCC_EA0_RDREQ_sum',0)/1e6)
PY
