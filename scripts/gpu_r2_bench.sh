# Round-2: the new headline bench (all-sources strong scaling) + side benches.
set -o pipefail
T=${TAG:-r2s11}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
cut -c1-2500 $O/bench.json
timeout -k 10 500 python -u bench.py --topology fabric100k-w --steps 2 --warmup 1 > $O/bench_w.json 2> $O/bench_w.err || { echo BW_FAIL; tail -20 $O/bench_w.err; exit 1; }
cut -c1-1200 $O/bench_w.json
timeout -k 10 600 python -u bench.py --topology mesh1m --steps 1 --warmup 1 > $O/bench_m.json 2> $O/bench_m.err || { echo BM_FAIL; tail -20 $O/bench_m.err; exit 1; }
cut -c1-1200 $O/bench_m.json
TAG=$T/prof bash scripts/gpu_r2_classprof.sh || exit 1
