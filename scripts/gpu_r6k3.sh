#!/bin/bash
# round 6: KSP2 A/B (gpu_r6k.sh), then the KSP2 parity tests under $KTEST env
set -u
OUT=gpurun_out/r6_${1:-k7}; mkdir -p $OUT; export TMPDIR=/tmp
bash scripts/gpu_r6k.sh ${1:-k7} || exit 1
timeout -k 10 500 env ${KTEST:-} python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_shard.py -m gpu -k "ksp" > $OUT/ksp_tests.log 2>&1 || { tail -30 $OUT/ksp_tests.log; exit 1; }
tail -2 $OUT/ksp_tests.log
