#!/bin/bash
# round 6: aligned sweep rows -- derive / sweep parity, then the headline with an in-process A/B
set -u
OUT=gpurun_out/r6_${1:-f1}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_sweep.py tests/test_gpu_derive.py tests/test_gpu_multi.py > $OUT/tests.log 2>&1 \
  || { tail -n 40 $OUT/tests.log; exit 1; }
tail -n 2 $OUT/tests.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --ab "${AB:-OSPF_SWEEP_ROW_PITCH=V}" \
  > $OUT/bench.json 2> $OUT/bench.err || { tail -n 30 $OUT/bench.err; exit 1; }
python - <<PY
import json
d = json.load(open("$OUT/bench.json"))
r = d["roofline"]
print(d["value"], d["ms_per_step"], "parity", (d.get("parity_vs_cpu_sample") or {}).get("equal"))
for u in r["launches"]: print(u["launch"], u["isolated_launch_ms"], u["frac"])
print("probe", {k: v for k, v in r.get("store_probe", {}).items() if k.endswith("GBs")}, r.get("frac_of_box_store_rate"))
for a in r.get("ab", []): print(a)
PY
