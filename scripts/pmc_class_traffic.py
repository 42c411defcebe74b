#!/usr/bin/env python3
"""HBM traffic of one root class per launch: rocprofv3 --pmc FETCH_SIZE and
WRITE_SIZE passes (separate: 3 + 2 > 4 TCC slots on gfx950) over
`bench.py --class-only CAP --reps R` (the class alone, R launches on one
stream), summed over every engine kernel (a class launch is a sequence of
kernels) and divided by R. MI355X_MICROARCH.md §HBM: FETCH_SIZE reads half
the bytes of a wide coalesced stream on gfx950 -> x2; WRITE_SIZE as is.

Usage: pmc_class_traffic.py FETCH_DIR WRITE_DIR LAUNCHES ROOTS KEY OUT_JSON
(OUT_JSON is updated in place: one entry per KEY, e.g. variant5_cap8)."""
import csv
import glob
import json
import os
import sys


def total(dirpath, counter):
    s, n = 0.0, 0
    for p in glob.glob(os.path.join(dirpath, "**", "*counter_collection.csv"), recursive=True):
        with open(p) as f:
            for r in csv.DictReader(f):
                if r.get("Counter_Name") == counter and "ospf::" in r.get("Kernel_Name", ""):
                    s += float(r["Counter_Value"])
                    n += 1
    return s, n


def main():
    fetch_dir, write_dir, launches, roots, key, out = sys.argv[1:7]
    launches, roots = int(launches), int(roots)
    fk, nf = total(fetch_dir, "FETCH_SIZE")
    wk, nw = total(write_dir, "WRITE_SIZE")
    res = json.load(open(out)) if os.path.exists(out) else {}
    per = (2 * fk + wk) * 1024 / launches
    res[key] = {"roots_per_launch": roots, "launches": launches,
                "fetch_size_kib_per_launch": fk / launches,
                "write_size_kib_per_launch": wk / launches,
                "hbm_bytes_per_launch": int(round(per)),
                "hbm_bytes_per_root": int(round(per / roots)),
                "dispatches": [nf, nw]}
    with open(out, "w") as fo:
        json.dump(res, fo, indent=1, sort_keys=True)
    print(json.dumps(res[key]))


if __name__ == "__main__":
    main()
