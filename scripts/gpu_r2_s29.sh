set -o pipefail
T=${TAG:-r2s29}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_derive.py > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 600 python -u bench.py --steps 10 --warmup 2 > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -30 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],[(u['launch'],u['isolated_launch_ms'],u['frac']) for u in d['roofline']['launches']], d['parity_vs_cpu_sample'])"
timeout -k 10 600 python -u scripts/prod_callstack.py > $O/prod_callstack.json 2> $O/prod_callstack.err || { echo PROD_FAIL; tail -30 $O/prod_callstack.err; exit 1; }
cat $O/prod_callstack.json
timeout -k 10 500 python -u scripts/bench_ksp2.py --steps 3 > $O/ksp.json 2> $O/ksp.err || { echo KSP_FAIL; tail -20 $O/ksp.err; exit 1; }
cat $O/ksp.json
