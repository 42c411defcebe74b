#!/bin/bash
# round-5 unit profiles of the headline sweep: kernel trace, FETCH / WRITE
# PMC passes, SQ pass -> units_trace.json, pmc_traffic.json, pmc_sq.json;
# PROF_ARGS selects another bench configuration (e.g. the M1M part)
set -u
OUT=gpurun_out/r5_${1:-e1}; mkdir -p $OUT; export TMPDIR=/tmp
A="${PROF_ARGS:-}"
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d "$OUT/utrace" -o run --output-format csv -- \
  python bench.py --steps 5 --warmup 1 --no-cpu --iso-reps 3 $A > "$OUT/utrace_bench.json" 2> "$OUT/utrace.err" || exit 1
i=0
for P in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $P -d "$OUT/upmc$i" -o run --output-format csv -- \
    python bench.py --steps 1 --warmup 0 --no-cpu --iso-reps 1 $A > "$OUT/upmc$i.json" 2> "$OUT/upmc$i.err" || exit 1
done
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY -d "$OUT/upmcsq" -o run --output-format csv -- \
  python bench.py --steps 1 --warmup 0 --no-cpu --iso-reps 1 $A > "$OUT/upmcsq.json" 2> "$OUT/upmcsq.err" || exit 1
python scripts/sweep_unit_stats.py --bench "$OUT/utrace_bench.json" --trace "$OUT/utrace" --reps 3 --out "$OUT/units_trace.json" &&
python scripts/sweep_unit_stats.py --bench "$OUT/upmc1.json" --pmc "$OUT/upmc1" "$OUT/upmc2" --reps 1 --out "$OUT/pmc_traffic.json" &&
python scripts/sweep_unit_stats.py --bench "$OUT/upmcsq.json" --pmc "$OUT/upmcsq" --reps 1 --out "$OUT/pmc_sq.json" > /dev/null
