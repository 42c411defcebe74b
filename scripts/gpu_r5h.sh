#!/bin/bash
# round-5 session H: sweep / derive / link-event parity after the parallel
# plan, plan phases, prod call stack (link / node events)
set -u
OUT=gpurun_out/r5_${1:-h1}; mkdir -p $OUT; export TMPDIR=/tmp
PYT="python -u -m pytest -x -q --timeout-method thread"
timeout -k 10 500 $PYT --timeout 300 tests/test_gpu_sweep.py tests/test_gpu_derive.py tests/test_gpu_link_events.py > $OUT/sweep.log 2>&1 || exit 1
OSPF_SWEEP_TIMING=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu --iso-reps 1 > $OUT/bench.json 2> $OUT/bench.err || exit 1
grep sweep_create $OUT/bench.err | tail -14
OSPF_SWEEP_TIMING=1 timeout -k 10 400 python scripts/prod_callstack.py --no-cpu > $OUT/prod.json 2> $OUT/prod.err || exit 1
grep -E "link_|node_" $OUT/prod.err | head -20
