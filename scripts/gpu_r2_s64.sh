set -o pipefail
O=gpurun_out/r2s64
mkdir -p $O
export TMPDIR=/tmp
for mode in batch derive; do
  timeout -k 10 300 python -u bench.py --topology grid31 --mode $mode --steps 60 --warmup 3 --no-cpu --iso-reps 1 > $O/b.json 2> $O/b.err || { echo BENCH_FAIL $mode; tail -20 $O/b.err; exit 1; }
  python -c "import json;d=json.load(open('$O/b.json'));print('$mode', d['value'], d['ms_per_step'], [(c.get('variant'), c.get('isolated_launch_ms')) for c in d['config']['root_classes']])"
done
