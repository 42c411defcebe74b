set -o pipefail
T=${TAG:-r2s37}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_derive.py tests/test_gpu_scale.py > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for env in "OSPF_LVX=0"; do
  env $env timeout -k 10 300 python3 scripts/exp_derive.py --reps 2 --check 64 > $O/exp.json 2> $O/exp.err || { echo EXP_FAIL; tail -5 $O/exp.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/exp.json'));print('$env', round(d['median_phase1_ms'],2), {k:round(v,2) for k,v in d['median_phase2_ms'].items()}, round(d['step_ms'],2), d['check_equal'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 scripts/exp_derive.py --reps 1 --check 0 > $O/kt.log 2>&1 || { echo KT_FAIL; tail -5 $O/kt.log; exit 1; }
python - <<PY
import csv,glob
rows=list(csv.DictReader(open(glob.glob('$O/kt/**/*kernel_stats.csv',recursive=True)[0])))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:12]:
    print(f"{float(r['TotalDurationNs'])/1e6/2:9.2f} ms/launch {int(r['Calls']):5d} {r['Name'][:70]}")
PY
