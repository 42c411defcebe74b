#!/bin/bash
# round 6: in-process A/B of env knobs on the headline bench (AB="K=V;K2=V2")
set -u
OUT=gpurun_out/r6_${1:-tw}; mkdir -p $OUT
timeout -k 10 500 python -u bench.py --steps 20 --warmup 3 --no-probe --cpu-sample 4 --ab "$AB" --ab-rounds 3 \
  > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python - <<PY
import json
d = json.load(open("$OUT/bench.json")); r = d["roofline"]
print(d["ms_per_step"], d["parity_vs_cpu_sample"]["equal"], [(u["launch"], u["isolated_launch_ms"]) for u in r["launches"]])
for a in r.get("ab", []): print(a)
PY
