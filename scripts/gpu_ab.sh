#!/bin/bash
# A/B of env knobs on the headline bench: gpu_ab.sh TAG base "K=V" ...
set -u
OUT=gpurun_out/r5_${1:-ab}; shift; mkdir -p $OUT; export TMPDIR=/tmp
for kv in "$@"; do
  E=""; [ "$kv" = base ] || E="$kv"
  timeout -k 10 300 env $E python bench.py --steps 20 --warmup 2 --cpu-sample 8 --iso-reps 1 > "$OUT/ab_$kv.json" 2> "$OUT/ab_$kv.err" || exit 1
  echo "$kv $(python -c "import json; d=json.load(open('$OUT/ab_$kv.json')); print(d['value'], d['ms_per_step'], d['parity_vs_cpu_sample']['equal'])")"
done
