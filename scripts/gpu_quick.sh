#!/bin/bash
# Quick GPU session: parity tests + per-class timings (+ optional extra command).
set -u
TAG=${1:-q}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; echo "pytest rc=$rc"
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 400 python scripts/exp_class.py --n 4096 ${EXP_ARGS:-} > "$OUT/exp.jsonl" 2> "$OUT/exp.err"
rc=$?; cat "$OUT/exp.jsonl"; echo "exp rc=$rc"
case $rc in 0) ;; *) exit $rc;; esac
if [ -n "${EXTRA:-}" ]; then bash -c "$EXTRA"; fi
exit 0
