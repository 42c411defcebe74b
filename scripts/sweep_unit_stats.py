#!/usr/bin/env python3
"""Per-launch-unit kernel time and HBM traffic of an all-sources sweep from
rocprofv3 output of `bench.py` (default sweep path).

bench.py calls ospf_sweep_profile(reps) after the timed steps: every launch
unit runs alone on its stream reps + 1 times, and the library queues one
`sweep_unit_mark_kernel` dispatch before each unit and one after the last
(openr_amd/csrc/engine/spf_sweep.hip). Dispatches between the k-th and the
(k+1)-th marker of the profile phase (the last units + 1 markers in dispatch
order) belong to unit k; the unit names and root counts come from the bench
JSON line (roofline.launches, in unit order).

  --trace DIR   rocprofv3 --kernel-trace --output-format csv output: per unit
                the summed kernel time per launch and the per-kernel split
                (compare with the HIP-event launch time in the bench line)
  --pmc DIR...  rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE, ...): per unit
                counters per launch; hbm_bytes = (2 x FETCH_SIZE + WRITE_SIZE)
                KiB (MI355X_MICROARCH.md: FETCH_SIZE reads 1/2 of the bytes of
                wide streaming reads on gfx950)
  --out FILE    merged JSON keyed by unit name (bench.py reads
                hbm_bytes_per_launch / roots_per_launch from
                profiles/<round>/pmc_traffic.json)
"""
import argparse
import collections
import csv
import glob
import json
import os
import re
import sys

MARK = "sweep_unit_mark_kernel"


def short(name):
    m = re.search(r"(\w+_kernel(?:<[^>]*>)?)", name)
    if m:
        return m.group(1)
    return "fillBuffer" if "fillBuffer" in name or "FillBuffer" in name else name[:60]


def rows_of(d, pattern):
    out = []
    for p in glob.glob(os.path.join(d, "**", pattern), recursive=True):
        with open(p) as f:
            out.extend(csv.DictReader(f))
    return out


def segments(disp, n_units):
    """{dispatch_id: record} -> list of n_units lists of records (profile phase)."""
    ids = sorted(disp)
    marks = [i for i in ids if MARK in disp[i]["name"]]
    if len(marks) < n_units + 1:
        raise SystemExit(f"found {len(marks)} unit markers, need {n_units + 1}")
    marks = marks[-(n_units + 1):]
    seg = []
    for k in range(n_units):
        lo, hi = marks[k], marks[k + 1]
        seg.append([disp[i] for i in ids if lo < i < hi])
    return seg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bench", required=True, help="bench.py JSON line (file)")
    ap.add_argument("--trace", default=None)
    ap.add_argument("--pmc", nargs="*", default=[])
    ap.add_argument("--reps", type=int, default=1, help="bench --iso-reps of the profiled run")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    with open(a.bench) as f:
        line = json.loads([ln for ln in f if ln.startswith("{")][-1])
    units = line["roofline"]["launches"]
    n = len(units)
    launches = a.reps + 1
    res = json.load(open(a.out)) if os.path.exists(a.out) else {}
    if a.trace:
        disp = {}
        for r in rows_of(a.trace, "*kernel_trace.csv"):
            disp[int(r["Dispatch_Id"])] = {
                "name": short(r["Kernel_Name"]),
                "ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                "t0": int(r["Start_Timestamp"]), "t1": int(r["End_Timestamp"])}
        for u, seg in zip(units, segments(disp, n)):
            per = collections.defaultdict(lambda: [0, 0])
            for r in seg:
                per[r["name"]][0] += 1
                per[r["name"]][1] += r["ns"]
            tot = sum(v[1] for v in per.values())
            span = (max(r["t1"] for r in seg) - min(r["t0"] for r in seg)) if seg else 0
            e = res.setdefault(u["launch"], {})
            e.update({
                "roots_per_launch": u["roots_per_launch"], "launches": launches,
                "kernel_sum_ms_per_launch": round(tot / launches / 1e6, 4),
                "span_ms_per_launch": round(span / launches / 1e6, 4),
                "hip_event_launch_ms": u["isolated_launch_ms"],
                "kernels": {k: {"dispatches_per_launch": v[0] / launches,
                                "ms_per_launch": round(v[1] / launches / 1e6, 4)}
                            for k, v in sorted(per.items(), key=lambda kv: -kv[1][1])},
                "trace_source": "rocprofv3 --kernel-trace (ospf_sweep_profile phase of bench.py)"})
    if a.pmc:
        disp = {}
        for d in a.pmc:
            for r in rows_of(d, "*counter_collection.csv"):
                key = (d, int(r["Dispatch_Id"]))
                rec = disp.setdefault(key, {"name": short(r["Kernel_Name"]), "c": {}})
                rec["c"][r["Counter_Name"]] = rec["c"].get(r["Counter_Name"], 0.0) + \
                    float(r["Counter_Value"])
        for d in a.pmc:  # every pass is a separate process: segment each alone
            sub = {i: v for (dd, i), v in disp.items() if dd == d}
            if not sub:
                continue
            for u, seg in zip(units, segments(sub, n)):
                e = res.setdefault(u["launch"], {})
                e["roots_per_launch"] = u["roots_per_launch"]
                e["launches"] = launches
                cs = e.setdefault("counters_per_launch", {})
                pk = e.setdefault("counters_by_kernel_per_launch", {})
                for r in seg:
                    for c, v in r["c"].items():
                        cs[c] = cs.get(c, 0.0) + v / launches
                        pk.setdefault(r["name"], {})
                        pk[r["name"]][c] = pk[r["name"]].get(c, 0.0) + v / launches
        for u in units:
            e = res.get(u["launch"], {})
            cs = e.get("counters_per_launch", {})
            if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
                hb = (2 * cs["FETCH_SIZE"] + cs["WRITE_SIZE"]) * 1024
                e["hbm_bytes_per_launch"] = int(round(hb))
                e["compulsory_bytes"] = u["compulsory_bytes"]
                e["traffic_over_compulsory"] = round(hb / u["compulsory_bytes"], 3)
                e["pmc_source"] = ("rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py "
                                   "(ospf_sweep_profile phase); hbm = (2 x FETCH_SIZE + "
                                   "WRITE_SIZE) KiB")
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    json.dump({k: {kk: v.get(kk) for kk in ("kernel_sum_ms_per_launch", "hip_event_launch_ms",
                                             "hbm_bytes_per_launch", "traffic_over_compulsory")}
               for k, v in res.items()}, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
