#!/bin/bash
# round-5 session D: KSP2 decremental phase clocks, prod call stack with the
# sweep-create phases, the captured-memset diagnostic at F100k-w
set -u
OUT=gpurun_out/r5_${1:-d1}; mkdir -p $OUT; export TMPDIR=/tmp
PYT="python -u -m pytest -x -q --timeout-method thread"
timeout -k 10 400 $PYT --timeout 200 tests/test_gpu_parity.py -k "ksp2 or ksp" > $OUT/t.log 2>&1 &&
OSPF_KSP_DEBUG=1 timeout -k 10 300 python scripts/bench_ksp2.py --no-cpu --steps 3 > $OUT/ksp.json 2> $OUT/ksp.err &&
OSPF_SWEEP_TIMING=1 timeout -k 10 400 python scripts/prod_callstack.py --no-cpu > $OUT/prod.json 2> $OUT/prod.err &&
timeout -k 10 500 python -u scripts/debug/replay_parity.py --topology fabric100k-w --variants memset > $OUT/memset.log 2>&1
