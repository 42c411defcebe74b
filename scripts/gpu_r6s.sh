#!/bin/bash
# round 6: the node-down sweep test, then the whole -m gpu suite and smoke
set -u
OUT=gpurun_out/r6_${1:-s1}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread \
  tests/test_gpu_link_events.py -k "node_down_up_sweep" > $OUT/nd.log 2>&1 || { tail -n 30 $OUT/nd.log; exit 1; }
tail -n 1 $OUT/nd.log
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests \
  > $OUT/suite.log 2>&1 || { tail -n 40 $OUT/suite.log; exit 1; }
tail -n 2 $OUT/suite.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
