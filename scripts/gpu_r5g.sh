#!/bin/bash
# round-5 session G: sweep-create phases at F100k, the publication -> CSR bench on the box's host
set -u
OUT=gpurun_out/r5_${1:-g1}; mkdir -p $OUT; export TMPDIR=/tmp
OSPF_SWEEP_TIMING=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu --iso-reps 1 > $OUT/bench.json 2> $OUT/bench.err || exit 1
grep sweep_create $OUT/bench.err | head -40
timeout -k 10 400 python scripts/bench_publication.py --reps 2 > $OUT/publication.json 2> $OUT/publication.err || exit 1
cat $OUT/publication.json
