#!/usr/bin/env python3
"""Sum rocprofv3 --pmc counter_collection.csv values per (kernel, counter)
over one or more output dirs; kernel names shortened to the function name.
Usage: pmc_by_kernel.py DIR [DIR ...] > out.json"""
import collections
import csv
import glob
import json
import os
import re
import sys


def short(name):
    m = re.search(r"(\w+_kernel(?:<[^>]*>)?)", name)
    return m.group(1) if m else name[:60]


def main():
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for d in sys.argv[1:]:
        for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(p) as f:
                for r in csv.DictReader(f):
                    k = short(r.get("Kernel_Name", ""))
                    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
                    disp[k].add(r.get("Dispatch_Id"))
    out = {k: dict(v, dispatches=len(disp[k])) for k, v in acc.items()}
    json.dump(out, sys.stdout, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
