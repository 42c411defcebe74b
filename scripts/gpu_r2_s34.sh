set -o pipefail
T=${TAG:-r2s34}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for opt in ""; do
  timeout -k 10 300 python3 scripts/exp_derive.py --reps 2 --check 16 $opt > $O/exp.json 2> $O/exp.err || { echo EXP_FAIL; tail -5 $O/exp.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/exp.json'));print('$opt', round(d['median_phase1_ms'],2), {k:round(v,2) for k,v in d['median_phase2_ms'].items()}, round(d['step_ms'],2), d['check_equal'])"
done
timeout -k 10 600 python -u bench.py --steps 5 --warmup 1 --no-cpu > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -30 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],[(u['launch'],u['isolated_launch_ms'],u['frac']) for u in d['roofline']['launches']])"
