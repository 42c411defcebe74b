#!/bin/bash
# round-5 session F: sweep / derive parity, F100k all-sources scale test, headline bench
set -u
OUT=gpurun_out/r5_${1:-f1}; mkdir -p $OUT; export TMPDIR=/tmp
PYT="python -u -m pytest -x -q --timeout-method thread"
timeout -k 10 500 $PYT --timeout 300 tests/test_gpu_sweep.py tests/test_gpu_derive.py > $OUT/sweep.log 2>&1 || exit 1
timeout -k 10 420 $PYT -s --timeout 400 tests/test_gpu_scale.py -k "f100k_all_sources" > $OUT/scale.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 2 --cpu-sample 8 --iso-reps 2 > $OUT/bench.json 2> $OUT/bench.err || exit 1
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['parity_vs_cpu_sample']['equal'], [(u['launch'], u['isolated_launch_ms']) for u in d['roofline'].get('launches', d['config']['root_classes'].get('launches', []))])"
