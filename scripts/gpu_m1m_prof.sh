#!/bin/bash
# M1M (weighted 1M-node mesh, sampled roots): kernel trace + HBM fetch / write
# passes of one timed step, to characterise the per-root Dial's bound.
set -u
OUT=gpurun_out/r3_m1m; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
  python bench.py --topology mesh1m --steps 1 --warmup 0 --no-cpu > "$OUT/trace_bench.json" 2> "$OUT/trace.err" || exit 1
for P in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $P -d "$OUT/pmc_$P" -o run --output-format csv -- \
    python bench.py --topology mesh1m --steps 1 --warmup 0 --no-cpu > "$OUT/pmc_$P.json" 2> "$OUT/pmc_$P.err" || exit 1
done
head -5 "$OUT/trace/run_kernel_stats.csv"
