#!/bin/bash
# round 6: sweep / derive / link-event / KSP2 parity after host-loop changes, then link-event re-sweep timing
set -u
OUT=gpurun_out/r6_${1:-w1}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_sweep.py tests/test_gpu_derive.py tests/test_gpu_link_events.py tests/test_gpu_multi.py tests/test_gpu_parity.py -k "sweep or derive or link or node or multi or ksp or load" > $OUT/tests.log 2>&1 \
  || { tail -n 30 $OUT/tests.log; exit 1; }
tail -n 1 $OUT/tests.log
OSPF_SWEEP_TIMING=1 timeout -k 10 400 python -u scripts/exp_link_event_sweep.py 6 > $OUT/ab.json 2> $OUT/ab.err || { tail -20 $OUT/ab.err; exit 1; }
cat $OUT/ab.json
grep "sweep_create plan " $OUT/ab.err | tail -4
