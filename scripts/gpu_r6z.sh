#!/bin/bash
# round 6 final, part A: the whole -m gpu suite, smoke, the default bench
set -u
OUT=gpurun_out/r6_${1:-z1}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests \
  > $OUT/suite.log 2>&1 || { tail -n 40 $OUT/suite.log; exit 1; }
tail -n 2 $OUT/suite.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -n 1 $OUT/smoke.log
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -n 20 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], d['parity_vs_cpu_sample']['equal'], r['frac'], r.get('frac_of_box_store_rate'))"
