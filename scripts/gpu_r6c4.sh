#!/bin/bash
# round 6: sweep / link-event parity after host-plan changes, then the production call stack
set -u
OUT=gpurun_out/r6_${1:-c4}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_sweep.py tests/test_gpu_derive.py tests/test_gpu_link_events.py tests/test_gpu_multi.py > $OUT/tests.log 2>&1 \
  || { tail -n 30 $OUT/tests.log; exit 1; }
tail -n 1 $OUT/tests.log
bash scripts/gpu_r6c2.sh ${1:-c4}
