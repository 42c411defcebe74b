#!/bin/bash
# twin levels prefetch A/B: derive parity, then units + bench per variant
set -u
OUT=gpurun_out/r5_${1:-k1}; mkdir -p $OUT; export TMPDIR=/tmp
PYT="python -u -m pytest -x -q --timeout-method thread"
timeout -k 10 500 $PYT --timeout 300 tests/test_gpu_sweep.py tests/test_gpu_derive.py > $OUT/sweep.log 2>&1 || { tail -n 30 $OUT/sweep.log; exit 1; }
tail -n 1 $OUT/sweep.log
for kv in base OSPF_TWIN_PREFETCH=1 base OSPF_TWIN_PREFETCH=1; do
  E=""; [ "$kv" = base ] || E="$kv"
  timeout -k 10 300 env $E python bench.py --steps 20 --warmup 2 --no-cpu --iso-reps 3 > $OUT/ab.json 2> $OUT/ab.err || exit 1
  python -c "import json; d=json.load(open('$OUT/ab.json')); print('$kv', d['value'], d['ms_per_step'], [(u['launch'], u['isolated_launch_ms']) for u in d['roofline']['launches'][:2]])"
done
