set -o pipefail
T=${TAG:-r2s30}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_derive.py tests/test_gpu_parity.py > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 600 python -u bench.py --steps 10 --warmup 2 > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -30 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],[(u['launch'],u['isolated_launch_ms'],u['frac']) for u in d['roofline']['launches']], d['parity_vs_cpu_sample'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 scripts/exp_derive.py --reps 1 --check 0 > $O/kt.log 2>&1 || { echo KT_FAIL; tail -5 $O/kt.log; exit 1; }
python - <<PY
import csv,glob
rows=list(csv.DictReader(open(glob.glob('$O/kt/**/*kernel_stats.csv',recursive=True)[0])))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:12]:
    print(f"{float(r['TotalDurationNs'])/1e6/2:9.2f} ms/launch {int(r['Calls']):5d} {r['Name'][:70]}")
PY
