#!/bin/bash
# round 6 final, part B: headline unit traces + PMC traffic + rocprofv3 stats,
# the KSP2 side bench with CPU baseline and parity, the production call stack
set -u
TAG=${1:-z2}; OUT=gpurun_out/r6_$TAG; mkdir -p $OUT; export TMPDIR=/tmp
STEPS="unitprof prof" bash scripts/gpu_r6.sh $TAG || exit 1
timeout -k 10 500 python -u scripts/bench_ksp2.py > $OUT/ksp2.json 2> $OUT/ksp2.err || { tail -20 $OUT/ksp2.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/ksp2.json')); print(d['value'], d['ms_per_step'], d.get('isolated_ms'), d['parity_vs_cpu_sample']['equal'])"
bash scripts/gpu_r6c2.sh $TAG
