set -o pipefail
T=${TAG:-r2s28}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u scripts/prod_callstack.py > $O/prod_callstack.json 2> $O/prod_callstack.err || { echo PROD_FAIL; tail -30 $O/prod_callstack.err; exit 1; }
cat $O/prod_callstack.json
timeout -k 10 500 python -u scripts/bench_ksp2.py --steps 3 > $O/ksp.json 2> $O/ksp.err || { echo KSP_FAIL; tail -20 $O/ksp.err; exit 1; }
cat $O/ksp.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 scripts/bench_ksp2.py --steps 1 --warmup 1 --iso-reps 1 --no-cpu > $O/kt.json 2> $O/kt.err || { echo KT_FAIL; tail -5 $O/kt.err; exit 1; }
python - <<PY
import csv,glob
rows=list(csv.DictReader(open(glob.glob('$O/kt/**/*kernel_stats.csv',recursive=True)[0])))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:10]:
    print(f"{float(r['AverageNs'])/1e6:9.3f} ms avg {int(r['Calls']):5d} {r['Name'][:70]}")
PY
