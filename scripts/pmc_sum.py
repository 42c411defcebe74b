#!/usr/bin/env python3
"""HBM bytes per launch of a multi-kernel engine call from two rocprofv3
--pmc passes (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950: 3 + 2
> 4 TCC slots): the sum over every dispatch of the engine's kernels (name
contains "spf_" or --match), divided by the number of calls the profiled
command made (--launches). MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB) counts
half the bytes of a wide coalesced stream on gfx950 -> x2 (an upper bound for
gathers); WRITE_SIZE (KiB) as is.

Usage: pmc_sum.py FETCH_DIR WRITE_DIR --launches N [--match S] [--extra k=v ...] > out.json
"""
import argparse
import csv
import glob
import json
import os


def total(dirpath, counter, match):
    s, n = 0.0, 0
    for p in glob.glob(os.path.join(dirpath, "**", "*counter_collection.csv"), recursive=True):
        with open(p) as f:
            for r in csv.DictReader(f):
                if r.get("Counter_Name") != counter or match not in r.get("Kernel_Name", ""):
                    continue
                s += float(r["Counter_Value"])
                n += 1
    return s, n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--launches", type=int, required=True)
    ap.add_argument("--match", default="spf_")
    ap.add_argument("--extra", nargs="*", default=[])
    a = ap.parse_args()
    fk, nf = total(a.fetch_dir, "FETCH_SIZE", a.match)
    wk, nw = total(a.write_dir, "WRITE_SIZE", a.match)
    out = {"fetch_size_kib_total": fk, "write_size_kib_total": wk, "dispatches": [nf, nw],
           "launches": a.launches,
           "hbm_bytes_per_launch": int(round((2 * fk + wk) * 1024 / max(1, a.launches))),
           "write_bytes_per_launch": int(round(wk * 1024 / max(1, a.launches))),
           "note": "FETCH_SIZE x2 (gfx950 wide-read correction) + WRITE_SIZE, summed over the "
                   "engine's dispatches, per call of the profiled command"}
    for kv in a.extra:
        k, v = kv.split("=", 1)
        out[k] = int(v) if v.isdigit() else v
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
