set -o pipefail
T=${TAG:-r2s32}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_derive.py tests/test_gpu_parity.py -k "derive or ksp or KSP or msbfs" > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 scripts/exp_derive.py --reps 1 --check 0 > $O/kt.log 2>&1 || { echo KT_FAIL; tail -5 $O/kt.log; exit 1; }
python - <<PY
import csv,glob
rows=list(csv.DictReader(open(glob.glob('$O/kt/**/*kernel_stats.csv',recursive=True)[0])))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:12]:
    print(f"{float(r['TotalDurationNs'])/1e6/2:9.2f} ms/launch {int(r['Calls']):5d} {r['Name'][:70]}")
PY
