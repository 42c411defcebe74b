#!/usr/bin/env python3
"""Multi-GPU readiness without the hardware: the F100k
all-sources sweep run as n_parts = 2 / 4 / 8 parts of the library's root
partition (ospf_sweep_opts.part / n_parts: pod blocks for racks and fabric
switches, plane blocks for spines, each part computing the rows of its
closure) on ONE GPU, part after part.

For every split: the union of the parts' digests must equal the single
sweep's (every root owned once, bit for bit); per part the roots it owns, the
rows it computes (closure overhead = rows / roots) and its isolated run time
(HIP-graph replays, median of --reps). The max part time is the PROJECTED
step of an N-GPU node -- unmeasured on N GPUs: it leaves out the RCCL digest
all-gather (24 B per root) and any per-device clock / HBM difference.

Usage: python scripts/parts_projection.py [--topology fabric100k] [--reps 10] > out.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402,F401  (one HIP runtime for torch and the engine)

from openr_amd import topology as T  # noqa: E402
from openr_amd.engine import Engine, Sweep  # noqa: E402
from openr_amd.linkstate import LinkState  # noqa: E402


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def timed_runs(sw, eng, reps):
    s = torch.cuda.current_stream()
    ms = []
    for k in range(reps + 1):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        sw.run(s.cuda_stream)
        b.record(s)
        b.synchronize()
        if k:
            ms.append(a.elapsed_time(b))
    eng.sync(s.cuda_stream)
    return float(np.median(ms)), float(np.min(ms))


def digests(sw, V):
    d = np.zeros((max(1, sw.n_roots), 3), np.uint64)
    sw._check(sw._L.ospf_sweep_digests_host(sw._h, d.ctypes.data))
    return sw.roots.copy(), d[: sw.n_roots]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--topology", default="fabric100k", choices=["fabric100k", "fabric10k",
                                                                 "fabric100k-w"])
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--parts", default="2,4,8")
    args = ap.parse_args()
    pods = 173 if args.topology == "fabric10k" else 1781
    st = T.fabric(pods=pods, planes=8, weighted_seed=7 if args.topology.endswith("-w") else None)
    ls = LinkState()
    ls.apply(st)
    csr = ls.csr()
    eng = Engine()
    eng.load(csr)
    V = eng.V
    sw = Sweep(eng)
    med, mn = timed_runs(sw, eng, args.reps)
    roots, d = digests(sw, V)
    full = np.zeros((V, 3), np.uint64)
    full[roots] = d
    out = {"topology": args.topology, "V": V, "mode": sw.mode,
           "single": {"roots": sw.n_roots, "rows": sw.n_rows, "ms_median": round(med, 3),
                      "ms_min": round(mn, 3), "spf_per_s": round(V / med * 1e3, 1)},
           "splits": {}}
    sw.close()
    log(f"single sweep: {med:.2f} ms, {out['single']['spf_per_s']:.0f} SPF/s")
    for n in [int(x) for x in args.parts.split(",")]:
        parts, union = [], np.zeros((V, 3), np.uint64)
        seen = np.zeros(V, np.int32)
        for i in range(n):
            t0 = time.time()
            p = Sweep(eng, part=i, n_parts=n)
            create_s = time.time() - t0
            med, mn = timed_runs(p, eng, args.reps)
            r, dd = digests(p, V)
            seen[r] += 1
            union[r] = dd
            parts.append({"part": i, "roots": p.n_roots, "rows": p.n_rows,
                          "closure_over_roots": round(p.n_rows / max(1, p.n_roots), 4),
                          "ms_median": round(med, 3), "ms_min": round(mn, 3),
                          "create_s": round(create_s, 2), "mode": p.mode})
            p.close()
            log(f"n={n} part {i}: {parts[-1]}")
        worst = max(x["ms_median"] for x in parts)
        out["splits"][str(n)] = {
            "parts": parts,
            "every_root_once": bool(np.all(seen == 1)),
            "union_equals_single": bool(np.array_equal(union, full)),
            "rows_total": int(sum(x["rows"] for x in parts)),
            "projected_step_ms": round(worst, 3),
            "projected_spf_per_s": round(V / worst * 1e3, 1),
            "projected_speedup": round(out["single"]["ms_median"] / worst, 3),
            "note": "PROJECTION, unmeasured on multiple GPUs: max over parts of each part's "
                    "isolated one-GPU run; excludes the RCCL all-gather of 24-B digests",
        }
        log(f"n={n}: projected {worst:.2f} ms, union == single: "
            f"{out['splits'][str(n)]['union_equals_single']}")
    eng.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
