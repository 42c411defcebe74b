#!/bin/bash
# round-5 session J: sweep / derive parity + headline bench (twin levels SWAR digest)
set -u
OUT=gpurun_out/r5_${1:-j1}; mkdir -p $OUT; export TMPDIR=/tmp
PYT="python -u -m pytest -x -q --timeout-method thread"
timeout -k 10 500 $PYT --timeout 300 tests/test_gpu_sweep.py tests/test_gpu_derive.py > $OUT/sweep.log 2>&1 || { tail -n 30 $OUT/sweep.log; exit 1; }
tail -n 1 $OUT/sweep.log
bash scripts/gpu_ab.sh ${1:-j1}ab base
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu --iso-reps 3 > $OUT/units.json 2> $OUT/units.err || exit 1
python -c "import json; d=json.load(open('$OUT/units.json')); print([(u['launch'], u['isolated_launch_ms']) for u in d['roofline'].get('launches', d['config']['root_classes'].get('launches', []))])"
