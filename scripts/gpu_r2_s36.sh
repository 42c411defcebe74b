set -o pipefail
T=${TAG:-r2s36}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 600 python -u bench.py --steps 20 --warmup 2 > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -30 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],[(u['launch'],u['isolated_launch_ms'],u['frac']) for u in d['roofline']['launches']], d['parity_vs_cpu_sample'], d['roofline']['step_frac'])"
