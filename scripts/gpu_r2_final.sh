set -o pipefail
O=gpurun_out/r2final
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -30 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['step_frac'],d['parity_vs_cpu_sample'],d['cpu_baseline']['value'])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu > $O/kt.log 2>&1 || { echo KT_FAIL; tail -5 $O/kt.log; exit 1; }
timeout -k 10 600 python -u scripts/bench_ksp2.py --steps 3 > $O/ksp.json 2> $O/ksp.err || { echo KSP_FAIL; tail -20 $O/ksp.err; exit 1; }
python -c "import json;d=json.load(open('$O/ksp.json'));print(d['value'],d['unit'],d.get('parity_vs_cpu_sample'))"
