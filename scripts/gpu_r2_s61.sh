set -o pipefail
O=gpurun_out/r2s61
mkdir -p $O
export TMPDIR=/tmp
for topo in fabric10k grid31 fabric10k-w; do
  timeout -k 10 400 python -u bench.py --topology $topo --steps 60 --warmup 3 > $O/bench_$topo.json 2> $O/bench_$topo.err || { echo BENCH_FAIL $topo; tail -20 $O/bench_$topo.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$topo.json'));print('$topo', d['value'], d['ms_per_step'], d['config']['mode'], d['roofline']['frac'], d['parity_vs_cpu_sample'], d['cpu_baseline']['value'] if d['cpu_baseline'] else None)"
done
