#!/usr/bin/env python3
"""Timeline of one ospf_ksp2_dev call from a rocprofv3 kernel trace of
scripts/bench_ksp2.py (the third call: warmup, timed, iso...).
Usage: python scripts/ksp_timeline.py <kernel_trace.csv> [call index]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ci = int(sys.argv[2]) if len(sys.argv) > 2 else 2
for r in rows:
    m = re.search(r"ospf::(?:\(anonymous namespace\)::)?(\w+)", r["Kernel_Name"])
    r["k"] = m.group(1) if m else r["Kernel_Name"][:20]
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
rows.sort(key=lambda r: r["s"])
big = max(int(r["Grid_Size_X"]) for r in rows if r["k"] == "ksp_trace_kernel")
starts = [i for i, r in enumerate(rows) if r["k"] == "ksp_trace_kernel" and int(r["Grid_Size_X"]) == big]
i0 = starts[ci]
i1 = starts[ci + 1] if ci + 1 < len(starts) else len(rows)
t0 = rows[i0 - 3]["s"]
seg = rows[i0 - 6:i1]
print("call span ms", round((max(r["e"] for r in seg) - t0) / 1e6, 3))
agg = {}
for r in seg:
    a = agg.setdefault(r["k"], [0, 0.0])
    a[0] += 1
    a[1] += (r["e"] - r["s"]) / 1e6
print({k: (v[0], round(v[1], 2)) for k, v in agg.items()})
for r in seg:
    if r["k"] in ("ksp_trace_kernel", "ksp_heavy_kernel", "msbfs_init_kernel"):
        print(f'{r["k"]:20s} {(r["s"] - t0) / 1e6:8.2f} {(r["e"] - t0) / 1e6:8.2f} grid {r["Grid_Size_X"]}')
# every kernel of the call: start / end / duration (ms from the call's start), queue
print("all kernels:")
for r in seg:
    q = r.get("Queue_Id") or r.get("Stream_Id") or "?"
    print(f'{(r["s"] - t0) / 1e6:8.3f} {(r["e"] - t0) / 1e6:8.3f} {(r["e"] - r["s"]) / 1e6:7.3f} q{q} {r["k"]}')
print("end", round((max(r["e"] for r in seg) - t0) / 1e6, 3))
