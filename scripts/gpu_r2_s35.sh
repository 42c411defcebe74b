set -o pipefail
T=${TAG:-r2s35}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_derive.py > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python3 scripts/exp_derive.py --reps 2 --check 64 > $O/exp.json 2> $O/exp.err || { echo EXP_FAIL; tail -5 $O/exp.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/exp.json'));print(round(d['median_phase1_ms'],2), {k:round(v,2) for k,v in d['median_phase2_ms'].items()}, round(d['step_ms'],2), d['check_equal'])"
