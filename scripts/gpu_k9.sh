#!/bin/bash
# KSP2 kernel timeline: rocprofv3 kernel trace of one bench_ksp2 step
set -u
OUT=gpurun_out/r5_${1:-k9}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python scripts/bench_ksp2.py --no-cpu --no-lfa --steps 1 --warmup 1 --iso-reps 1 > $OUT/kspp.json 2> $OUT/kspp.err
