#!/usr/bin/env python3
"""Per-launch HBM traffic of each engine kernel class from two rocprofv3 --pmc
passes (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950: 3 + 2 > 4 TCC
slots). Applies MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB) reads half the
bytes of a wide coalesced stream on gfx950 -> x2; WRITE_SIZE (KiB) as is.

Usage: pmc_traffic.py FETCH_DIR WRITE_DIR BENCH_JSON OUT_JSON
Kernels are matched to bench.py's root classes by launch geometry
(grid threads = roots_per_step x slices x block).
"""
import csv
import glob
import json
import os
import statistics
import sys


def load(dirpath, counter):
    rows = []
    for p in glob.glob(os.path.join(dirpath, "**", "*counter_collection.csv"), recursive=True):
        with open(p) as f:
            for r in csv.DictReader(f):
                if r.get("Counter_Name") != counter:
                    continue
                name = r.get("Kernel_Name", "")
                if "spf_" not in name:
                    continue
                grid = int(r.get("Grid_Size") or r.get("Grid_Size_X") or 0)
                rows.append((name, grid, float(r["Counter_Value"])))
    return rows


def main():
    fetch_dir, write_dir, bench_json, out = sys.argv[1:5]
    bench = json.loads(open(bench_json).read().strip().splitlines()[-1])
    classes = bench["config"]["root_classes"]
    fetch, write = load(fetch_dir, "FETCH_SIZE"), load(write_dir, "WRITE_SIZE")
    res = {}
    for c in classes:
        grid = c["roots_per_step"] * c["slices"] * c["block"]
        f = [v for _, g, v in fetch if g == grid]
        w = [v for _, g, v in write if g == grid]
        if not f or not w:
            continue
        fk, wk = statistics.median(f), statistics.median(w)
        res[f"variant{c['variant']}_W{c['nh_words']}"] = {
            "grid_threads": grid, "roots_per_launch": c["roots_per_step"],
            "fetch_size_kib_median": fk, "write_size_kib_median": wk,
            "hbm_bytes_per_launch": int(round((2 * fk + wk) * 1024)),
            "hbm_bytes_per_root": int(round((2 * fk + wk) * 1024 / c["roots_per_step"])),
            "dispatches": [len(f), len(w)],
        }
    with open(out, "w") as fo:
        json.dump(res, fo, indent=1, sort_keys=True)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
