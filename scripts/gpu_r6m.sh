#!/bin/bash
# round 6: KSP2 A/B (gpu_r6k.sh), KSP2 parity with the candidate knob, then
# the production call stack with load / snapshot laps
set -u
OUT=gpurun_out/r6_${1:-m1}; mkdir -p $OUT; export TMPDIR=/tmp
bash scripts/gpu_r6k.sh ${1:-m1} || exit 1
if [ -n "${KTEST:-}" ]; then
  timeout -k 10 400 env $KTEST python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -k "ksp" > $OUT/ksp_tests.log 2>&1 || { tail -30 $OUT/ksp_tests.log; exit 1; }
  tail -2 $OUT/ksp_tests.log
fi
PROD_TRACE_FILE=$OUT/prod_stall.txt timeout -k 10 500 python -u scripts/prod_callstack.py --no-cpu > $OUT/prod.json 2> $OUT/prod.err || { tail -20 $OUT/prod.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/prod.json')); print({k: v for k, v in d.items() if 'cold' in k or 'link_' in k and 'ms' in k})"
