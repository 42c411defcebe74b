#!/usr/bin/env python3
"""Per-kernel totals and the longest dispatches of a rocprofv3 kernel trace of
scripts/bench_ksp2.py. Usage: python scripts/ksp_dispatch.py <kernel_trace.csv>"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tot, cnt = {}, {}
for r in rows:
    k = r["Kernel_Name"].split("(")[0][-40:]
    dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot[k] = tot.get(k, 0) + dur
    cnt[k] = cnt.get(k, 0) + 1
    r["_k"], r["_d"] = k, dur
for k in sorted(tot, key=lambda k: -tot[k]):
    print(f"{k:42s} n={cnt[k]:6d} total_ms={tot[k]/1e3:9.2f}")
print("longest:")
for r in sorted(rows, key=lambda r: -r["_d"])[:12]:
    print(f'{r["_k"]:42s} grid={r["Grid_Size_X"]:>9s} dur_us={r["_d"]:9.1f}')
