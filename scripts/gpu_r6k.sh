#!/bin/bash
# round 6: KSP2 A/B of env knobs (one bench_ksp2 run each), decr stats on stderr
set -u
OUT=gpurun_out/r6_${1:-k1}; mkdir -p $OUT; export TMPDIR=/tmp
for kv in base ${AB:-}; do
  E=""; [ "$kv" = base ] || E="${kv//,/ }"
  timeout -k 10 300 env OSPF_KSP_DEBUG=${KDBG:-1} $E python -u scripts/bench_ksp2.py --steps 3 --warmup 1 --no-cpu --no-lfa ${KSP_ARGS:-} > $OUT/ksp_$kv.json 2> $OUT/ksp_$kv.err || { tail -20 $OUT/ksp_$kv.err; exit 1; }
  echo "$kv $(python -c "import json; d=json.load(open('$OUT/ksp_$kv.json')); print(d['ms_per_step'], d.get('isolated_ms'))") $(grep 'ksp2 decr' $OUT/ksp_$kv.err | tail -1 | sed 's/.*heavy block-ms/heavy block-ms/')"
done
