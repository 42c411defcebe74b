#!/bin/bash
# round 6: headline with the store probe + in-process leaf A/B (block order, chunk size)
set -u
OUT=gpurun_out/r6_${1:-a1}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 \
  --ab "OSPF_LEAF_GROUP_MAJOR=1;OSPF_LEAF_CTILES=20;OSPF_LEAF_GROUP_MAJOR=1,OSPF_LEAF_CTILES=20;OSPF_LEAF_GROUP_MAJOR=1,OSPF_LEAF_CTILES=98" \
  > $OUT/bench.json 2> $OUT/bench.err || { tail -n 30 $OUT/bench.err; exit 1; }
python - <<PY
import json
d = json.load(open("$OUT/bench.json"))
r = d["roofline"]
print(d["value"], d["ms_per_step"], "parity", (d.get("parity_vs_cpu_sample") or {}).get("equal"))
print("leaf", r["avg_launch_ms"], r["frac"], "probe", json.dumps(r.get("store_probe")))
for a in r.get("ab", []): print(a)
PY
