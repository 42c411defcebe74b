#!/bin/bash
# KSP2 A/B: parity subset, then bench_ksp2 (decremental phase clocks) per knob
set -u
OUT=gpurun_out/r5_${1:-k8}; mkdir -p $OUT; export TMPDIR=/tmp
shift
PYT="python -u -m pytest -x -q --timeout-method thread"
timeout -k 10 400 $PYT --timeout 200 tests/test_gpu_parity.py -k "ksp2 or ksp" > $OUT/t.log 2>&1 || exit 1
if [ -n "${FULL:-}" ]; then
  OSPF_KSP_DEBUG=1 timeout -k 10 420 $PYT -s --timeout 400 tests/test_gpu_scale.py -k "role_stratified" > $OUT/t2.log 2>&1 || exit 1
fi
for kv in "$@"; do
  E=""; [ "$kv" = base ] || E="$kv"
  OSPF_KSP_DEBUG=1 timeout -k 10 300 env $E python scripts/bench_ksp2.py --no-cpu --no-lfa --steps 3 > $OUT/ksp_$kv.json 2> $OUT/ksp_$kv.err || exit 1
  echo "$kv $(python -c "import json; d=json.load(open('$OUT/ksp_$kv.json')); print(d['ms_per_step'], d['isolated_ms'])") $(tail -n 1 $OUT/ksp_$kv.err)"
done
