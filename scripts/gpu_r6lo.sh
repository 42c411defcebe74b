#!/bin/bash
# round 6: sweep tests after the leaf-order pick, then the in-process A/B
set -u
OUT=gpurun_out/r6_${1:-lo}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sweep.py tests/test_gpu_multi.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
OSPF_SWEEP_TIMING=1 AB="OSPF_LEAF_NO_AUTO=1;OSPF_LEAF_GROUP_MAJOR=1" bash scripts/gpu_r6tw.sh ${1:-lo} || exit 1
grep "leaf order" gpurun_out/r6_${1:-lo}/bench.err | head -8
