set -o pipefail
O=gpurun_out/r2s62
mkdir -p $O
export TMPDIR=/tmp
for topo in grid31 fabric10k fabric100k; do
  for gm in off on; do
    timeout -k 10 400 python -u bench.py --topology $topo --steps 30 --warmup 2 --graph $gm --no-cpu --iso-reps 1 > $O/b.json 2> $O/b.err || { echo BENCH_FAIL $topo $gm; tail -20 $O/b.err; exit 1; }
    python -c "import json;d=json.load(open('$O/b.json'));print('$topo', '$gm', d['value'], d['ms_per_step'], d['config']['root_classes'][0].get('hip_graph'))"
  done
done
timeout -k 10 300 python -u bench.py --topology fabric10k --steps 10 --warmup 2 --graph on > $O/b.json 2> $O/b.err || { echo BENCH_FAIL parity; tail -20 $O/b.err; exit 1; }
python -c "import json;d=json.load(open('$O/b.json'));print('parity', d['value'], d['parity_vs_cpu_sample'])"
