set -o pipefail
O=gpurun_out/r2s50
mkdir -p $O
export TMPDIR=/tmp
for env in "OPENR_WCOVER_KEY=last" "OPENR_WCOVER_KEY=first"; do
  env $env timeout -k 10 400 python -u bench.py --topology fabric100k-w --steps 3 --warmup 1 --no-cpu --iso-reps 2 > $O/b.json 2> $O/b.err || { echo BENCH_FAIL; tail -30 $O/b.err; exit 1; }
  python -c "import json;d=json.load(open('$O/b.json'));print('$env', d['value'],d['ms_per_step'],[(u['launch'],u['isolated_launch_ms']) for u in d['roofline']['launches']])"
done
