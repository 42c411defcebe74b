#!/bin/bash
# the whole -m gpu suite (as the driver runs it) + smoke()
set -u
OUT=gpurun_out/r5_${1:-s1}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 1050 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/suite.log 2>&1 || { tail -n 30 $OUT/suite.log; exit 1; }
tail -n 3 $OUT/suite.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -n 20 $OUT/smoke.log; exit 1; }
tail -n 1 $OUT/smoke.log
