#!/bin/bash
# round 6: production call stack A at F100k (cold / warm / events), progress on stderr
set -u
OUT=gpurun_out/r6_${1:-c2}; mkdir -p $OUT; export TMPDIR=/tmp
PROD_TRACE_FILE=$OUT/prod_stall.txt timeout -k 10 600 python -u scripts/prod_callstack.py --no-cpu > $OUT/prod.json 2> $OUT/prod.err || { tail -20 $OUT/prod.err; exit 1; }
grep -v "^\[" $OUT/prod.err | tail -12
