set -o pipefail
T=${TAG:-r2s33}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for opt in "" "--no-digest" "--no-dist" "--no-digest --no-dist"; do
  timeout -k 10 300 python3 scripts/exp_derive.py --reps 2 --check 0 $opt > $O/exp.json 2> $O/exp.err || { echo EXP_FAIL; tail -5 $O/exp.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/exp.json'));print('$opt', round(d['median_phase1_ms'],2), {k:round(v,2) for k,v in d['median_phase2_ms'].items()}, round(d['step_ms'],2))"
done
