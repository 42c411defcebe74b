#!/bin/bash
# One gpurun session: GPU parity tests, a short bench, a rocprofv3 kernel-trace
# summary. Stops at the first GPU fault / abort / timeout (exit 124,134,137,139),
# continues past plain test failures (exit 1) so the bench still runs.
# Usage: bash scripts/gpu_session.sh [tag] [pytest-args...]
set -u
TAG=${1:-s1}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }

echo "== pytest -m gpu" | tee -a "$OUT/session.log"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread "$@" \
  > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc" | tee -a "$OUT/session.log"; tail -5 "$OUT/pytest_gpu.log"
if fatal $rc; then echo "fatal pytest exit; stopping"; exit $rc; fi

echo "== bench" | tee -a "$OUT/session.log"
timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc" | tee -a "$OUT/session.log"; cat "$OUT/bench.json"; tail -3 "$OUT/bench.err"
if fatal $rc; then exit $rc; fi
if [ -n "${BENCH2_ARGS:-}" ]; then
  timeout -k 10 400 python -u bench.py --no-cpu $BENCH2_ARGS > "$OUT/bench2.json" 2> "$OUT/bench2.err"
  rc=$?; echo "bench2 rc=$rc" | tee -a "$OUT/session.log"; cat "$OUT/bench2.json"
  if fatal $rc; then exit $rc; fi
fi

echo "== rocprofv3 kernel trace" | tee -a "$OUT/session.log"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
  -- python3 bench.py --steps 3 --warmup 1 --no-cpu > "$OUT/prof_bench.json" 2> "$OUT/prof.err"
rc=$?; echo "rocprof rc=$rc" | tee -a "$OUT/session.log"
find "$OUT/prof" -name "*kernel_stats.csv" -exec cat {} \; | head -20
if [ -n "${PMC:-}" ]; then
  echo "== rocprofv3 PMC passes" | tee -a "$OUT/session.log"
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv \
    -- python3 bench.py --steps 2 --warmup 1 --no-cpu > "$OUT/pmc_fetch.json" 2> "$OUT/pmc_fetch.err"
  rc=$?; echo "pmc fetch rc=$rc" | tee -a "$OUT/session.log"; if fatal $rc; then exit $rc; fi
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv \
    -- python3 bench.py --steps 2 --warmup 1 --no-cpu > "$OUT/pmc_write.json" 2> "$OUT/pmc_write.err"
  rc=$?; echo "pmc write rc=$rc" | tee -a "$OUT/session.log"; if fatal $rc; then exit $rc; fi
  python3 scripts/pmc_traffic.py "$OUT/pmc_fetch" "$OUT/pmc_write" "$OUT/pmc_fetch.json" "$OUT/pmc_traffic.json" || true
fi
exit 0
