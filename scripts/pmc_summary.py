#!/usr/bin/env python3
"""Per-dispatch PMC summary of scripts/pmc_passes.sh output: for each pass's
counter_collection.csv, the counters of the last N dispatches matching a
kernel substring. Usage: python scripts/pmc_summary.py <outdir> [substr] [N]"""
import collections
import csv
import glob
import sys

out = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else "msbfs"
N = int(sys.argv[3]) if len(sys.argv) > 3 else 30
per = collections.OrderedDict()
for f in sorted(glob.glob(f"{out}/p*/**/*counter_collection.csv", recursive=True)):
    rows = [r for r in csv.DictReader(open(f)) if sub in r["Kernel_Name"]]
    disp = collections.OrderedDict()
    for r in rows:
        d = disp.setdefault(r["Dispatch_Id"], {"k": r["Kernel_Name"], "grid": r.get("Grid_Size", "")})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    keys = list(disp.keys())[-N:]
    for i, k in enumerate(keys):
        per.setdefault(i, {}).update(disp[k])
for i, d in per.items():
    name = d.pop("k")
    short = next((s for s in ("init", "level", "settle", "final", "digest") if s in name), name[:20])
    d.pop("grid", None)
    print(short, " ".join(f"{k}={v:.3g}" for k, v in d.items()))
