#!/bin/bash
# round-5 session C: slot sharding tests, the captured-memset diagnostic
# (DESIGN §3), then session B (sweep parity, headline A/B, KSP2)
set -u
OUT=gpurun_out/r5_${1:-c1}; mkdir -p $OUT; export TMPDIR=/tmp
PYT="python -u -m pytest -x -q --timeout-method thread"
timeout -k 10 300 $PYT --timeout 200 tests/test_gpu_shard.py > $OUT/shard.log 2>&1 || exit 1
timeout -k 10 400 python -u scripts/debug/replay_parity.py --topology fabric10k-w --variants memset,base,memsetoff > $OUT/memset.log 2>&1 || exit 1
bash scripts/gpu_r5b.sh ${1:-c1}
