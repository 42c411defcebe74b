#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace of the multi-source BFS: per dispatch
(kernel, grid, duration), for the last N dispatches. Usage:
  python scripts/trace_levels.py gpurun_out/<tag>/run_kernel_trace.csv [N]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 60
tot = {}
for r in rows:
    k = r["Kernel_Name"]
    short = next((s for s in ("init", "level", "settle", "final", "rows", "digest", "fill", "spf_bfs")
                  if s in k.lower()), k[:24])
    dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot[short] = tot.get(short, 0) + dur
    r["_s"], r["_d"] = short, dur
for r in rows[-n:]:
    print(f'{r["_s"]:8s} grid={r["Grid_Size_X"]:>9s} dur_us={r["_d"]:9.1f}')
print({k: round(v, 1) for k, v in tot.items()})
