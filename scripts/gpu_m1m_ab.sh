#!/bin/bash
# M1M part A/B of env knobs: gpu_m1m_ab.sh TAG base "K=V" ...
set -u
OUT=gpurun_out/r5_${1:-m1}; shift; mkdir -p $OUT; export TMPDIR=/tmp
for kv in "$@"; do
  E=""; [ "$kv" = base ] || E="$kv"
  timeout -k 10 400 env $E python bench.py --topology mesh1m --steps 3 --warmup 1 --no-cpu --iso-reps 1 > "$OUT/ab_$kv.json" 2> "$OUT/ab_$kv.err" || exit 1
  echo "$kv $(python -c "import json; d=json.load(open('$OUT/ab_$kv.json')); print(d['value'], d['ms_per_step'], d.get('parity_vs_cpu_sample'))")"
done
