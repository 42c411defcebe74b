#!/bin/bash
# round-5 session B: sweep parity after the fused twin dist rows, headline A/B,
# KSP2 decremental reruns (tests, F100k parity, profile, bench), prod call stack
set -u
OUT=gpurun_out/r5_${1:-b1}; mkdir -p $OUT; export TMPDIR=/tmp
PYT="python -u -m pytest -x -q --timeout-method thread"
timeout -k 10 500 $PYT --timeout 300 tests/test_gpu_sweep.py tests/test_gpu_derive.py > $OUT/sweep.log 2>&1 || exit 1
timeout -k 10 420 $PYT -s --timeout 400 tests/test_gpu_scale.py -k "f100k_all_sources" > $OUT/scale.log 2>&1 || exit 1
for kv in base OSPF_TWIN_DIST_IN_LEVELS=1; do
  E=""; [ "$kv" = base ] || E="$kv"
  timeout -k 10 300 env $E python bench.py --steps 20 --warmup 2 --cpu-sample 8 --iso-reps 2 > $OUT/ab_$kv.json 2> $OUT/ab_$kv.err || exit 1
  python -c "import json; d=json.load(open('$OUT/ab_$kv.json')); print('$kv', d['value'], d['ms_per_step'], d['parity_vs_cpu_sample']['equal'])"
done
bash scripts/gpu_k6.sh ${1:-b1}k
