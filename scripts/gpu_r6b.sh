#!/bin/bash
# round 6: new GPU tests (degrade, counters, teardown) + neighbours
set -u
OUT=gpurun_out/r6_${1:-b1}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_degrade.py tests/test_gpu_link_events.py tests/test_gpu_routes.py > $OUT/tests.log 2>&1 \
  || { tail -n 40 $OUT/tests.log; exit 1; }
tail -n 3 $OUT/tests.log
