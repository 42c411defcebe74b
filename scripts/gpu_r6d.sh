#!/bin/bash
# round 6: in-process A/B of the captured seed-BFS depth, then the sweep GPU tests
set -u
OUT=gpurun_out/r6_${1:-d1}; mkdir -p $OUT
AB="OSPF_SWEEP_FULL_DEPTH=1" bash scripts/gpu_r6tw.sh ${1:-d1} || exit 1
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread \
  tests/test_gpu_sweep.py tests/test_gpu_link_events.py tests/test_gpu_degrade.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
