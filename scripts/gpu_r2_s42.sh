set -o pipefail
T=${TAG:-r2s42}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for env in "OSPF_WD_GROUP=8" "OSPF_WD_GROUP=4" "OSPF_WD_GROUP=16" "OSPF_WD_GROUP=2"; do
  env $env timeout -k 10 400 python -u bench.py --topology fabric100k-w --steps 2 --warmup 1 --no-cpu --iso-reps 1 > $O/b.json 2> $O/b.err || { echo BENCH_FAIL; tail -30 $O/b.err; exit 1; }
  python -c "import json;d=json.load(open('$O/b.json'));print('$env', d['value'],d['ms_per_step'],[(u['launch'],u['isolated_launch_ms']) for u in d['roofline']['launches']])"
done
