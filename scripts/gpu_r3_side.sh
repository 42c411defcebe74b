#!/bin/bash
# Round-3 side measurements: production call stack (ingest, getSpfResult
# after an event), weighted F100k sweep, M1M sampled roots, KSP2 + LFA.
set -u
OUT=gpurun_out/r3_side${1:-}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/prod_callstack.py > "$OUT/prod_callstack.json" 2> "$OUT/prod_callstack.err" || { tail -20 "$OUT/prod_callstack.err"; exit 1; }
tail -c 1500 "$OUT/prod_callstack.json"; echo
timeout -k 10 400 python -u bench.py --topology fabric100k-w --steps 5 > "$OUT/bench_fabric100k_w.json" 2> "$OUT/bench_w.err" || { tail -20 "$OUT/bench_w.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_fabric100k_w.json')); print('w', d['value'], d['ms_per_step'], d['parity_vs_cpu_sample']['equal'])"
timeout -k 10 400 python -u bench.py --topology mesh1m --steps 2 --warmup 1 > "$OUT/bench_mesh1m.json" 2> "$OUT/bench_m.err" || { tail -20 "$OUT/bench_m.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_mesh1m.json')); print('m1m', d['value'], d['ms_per_step'], d['parity_vs_cpu_sample']['equal'])"
timeout -k 10 400 python -u scripts/bench_ksp2.py > "$OUT/bench_ksp2.json" 2> "$OUT/bench_ksp2.err" || { tail -20 "$OUT/bench_ksp2.err"; exit 1; }
tail -c 600 "$OUT/bench_ksp2.json"; echo
