set -o pipefail
T=${TAG:-r2s39}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_derive.py tests/test_gpu_multirank.py > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for env in "OSPF_LVX=0" "OSPF_MS_PUSH_DIV=8" "OSPF_MS_PUSH_DIV=32"; do
  env $env timeout -k 10 300 python3 scripts/exp_derive.py --reps 3 --check 32 > $O/exp.json 2> $O/exp.err || { echo EXP_FAIL; tail -5 $O/exp.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/exp.json'));print('$env', [round(x,2) for x in d['phase1_ms']], d['check_equal'])"
done
timeout -k 10 600 python -u bench.py --steps 20 --warmup 2 --no-cpu > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -30 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],[(u['launch'],u['isolated_launch_ms'],u['frac']) for u in d['roofline']['launches']], d['roofline']['step_frac'])"
