#!/bin/bash
# round 6: KSP2 kernel timelines (rocprofv3 kernel trace of bench_ksp2) for env variants
set -u
OUT=gpurun_out/r6_${1:-t1}; mkdir -p $OUT; cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for kv in base ${AB:-}; do
  E=""; [ "$kv" = base ] || E="${kv//,/ }"
  D=$OUT/tr_$kv
  timeout -k 10 300 env $E rocprofv3 --kernel-trace -d $D -o run --output-format csv -- python3 scripts/bench_ksp2.py --steps 1 --warmup 1 --iso-reps 1 --no-cpu --no-lfa > $D.json 2> $D.err || { tail -20 $D.err; exit 1; }
  f=$(find $D -name "*kernel_trace.csv" | head -1)
  python3 scripts/ksp_timeline.py "$f" 1 > $OUT/timeline_$kv.txt 2>&1 || true
  echo "== $kv"; head -3 $OUT/timeline_$kv.txt
done
