#!/bin/bash
# round 6: headline unit traces + PMC traffic (gpu_r6.sh unitprof), the
# rocprofv3 --stats summary of a short bench, then the default bench
set -u
TAG=${1:-p1}
STEPS="unitprof prof bench" BENCH_ARGS="${BENCH_ARGS:-}" bash scripts/gpu_r6.sh $TAG
