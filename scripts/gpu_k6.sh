#!/bin/bash
# KSP2 decremental reruns + link / node events: tests, F100k parity, profile, bench
set -u
OUT=gpurun_out/r5_${1:-k6}; mkdir -p $OUT; export TMPDIR=/tmp
PYT="python -u -m pytest -x -q --timeout-method thread"
timeout -k 10 400 $PYT --timeout 200 tests/test_gpu_parity.py -k "ksp2 or ksp" > $OUT/t.log 2>&1 &&
timeout -k 10 400 $PYT --timeout 200 tests/test_gpu_link_events.py > $OUT/t1.log 2>&1 &&
OSPF_KSP_DEBUG=1 timeout -k 10 420 $PYT -s --timeout 400 tests/test_gpu_scale.py -k "role_stratified" > $OUT/t2.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python scripts/bench_ksp2.py --no-cpu --no-lfa --steps 2 --warmup 1 --iso-reps 1 > $OUT/kspp.json 2> $OUT/kspp.err &&
OSPF_KSP_DEBUG=1 timeout -k 10 300 python scripts/bench_ksp2.py --no-cpu --steps 5 > $OUT/ksp.json 2> $OUT/ksp.err
[ $? -eq 0 ] && OSPF_SWEEP_TIMING=1 timeout -k 10 400 python scripts/prod_callstack.py > $OUT/prod.json 2> $OUT/prod.err
