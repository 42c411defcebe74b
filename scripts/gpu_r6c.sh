#!/bin/bash
# round 6: best-route selection + multi-area on the engine + reference fixtures on the GPU
set -u
OUT=gpurun_out/r6_${1:-c1}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_routes.py tests/test_host_multiarea.py tests/test_gpu_degrade.py \
  "tests/test_gpu_parity.py::test_reference_fixture_on_gpu" > $OUT/tests.log 2>&1 \
  || { tail -n 40 $OUT/tests.log; exit 1; }
tail -n 3 $OUT/tests.log
