#!/bin/bash
# KSP2 HBM traffic: two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) over
# one bench_ksp2 step (3 KSP2 launches: warmup-free step + 2 isolated), summed
set -u
OUT=gpurun_out/r5_${1:-kpmc}; mkdir -p $OUT; export TMPDIR=/tmp
i=0
for P in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P -d "$OUT/kpmc$i" -o run --output-format csv -- \
    python scripts/bench_ksp2.py --steps 1 --warmup 0 --iso-reps 1 --no-cpu --no-lfa > "$OUT/kpmc$i.json" 2> "$OUT/kpmc$i.err" || exit 1
done
ND=$(python -c "import json; print(json.load(open('$OUT/kpmc1.json'))['roofline']['destinations_per_launch'])")
python scripts/pmc_sum.py "$OUT/kpmc1" "$OUT/kpmc2" --launches 3 --match "ospf::" --extra destinations_per_launch=$ND > "$OUT/ksp2_pmc.json"
