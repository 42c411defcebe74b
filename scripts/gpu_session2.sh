#!/bin/bash
# GPU session for the multi-source engine: parity tests, the bench (with the
# CPU baseline), a rocprofv3 kernel-trace summary of the bench, and per-class
# PMC traffic (each class alone via exp_class, FETCH_SIZE and WRITE_SIZE in
# separate passes). Stops at the first GPU fault / abort / timeout.
# Usage: bash scripts/gpu_session2.sh TAG  (env: BENCH_ARGS, CLASSES="1:3501 3:583 56:12")
set -u
TAG=${1:-s}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest_gpu.log"
if fatal $rc; then exit $rc; fi
timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; cat "$OUT/bench.json"; if fatal $rc; then exit $rc; fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
  -- python3 bench.py --steps 5 --warmup 1 --no-cpu > "$OUT/prof_bench.json" 2> "$OUT/prof.err"
rc=$?; echo "rocprof rc=$rc"; if fatal $rc; then exit $rc; fi
for c in ${CLASSES:-1:3501 3:583 56:12}; do
  W=${c%%:*}; N=${c##*:}
  for P in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $P -d "$OUT/pmc_W${W}_$P" -o run --output-format csv \
      -- python3 scripts/exp_class.py --W $W --n $N --reps 2 ${EXP_ORDER:-} > "$OUT/pmc_W${W}_$P.log" 2>&1
    rc=$?; echo "pmc W$W $P rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
  done
  python3 scripts/pmc_class_traffic.py "$OUT/pmc_W${W}_FETCH_SIZE" "$OUT/pmc_W${W}_WRITE_SIZE" 3 $N \
    variant5_W$W "$OUT/pmc_traffic.json"
done
exit 0
