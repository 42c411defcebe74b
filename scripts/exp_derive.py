#!/usr/bin/env python3
"""Derive-mode experiment at F100k: phase 1 (levels of all roots) and phase 2
(next hops per width class) timed with HIP events on one stream, checked
against the per-batch engine path on sampled roots."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from openr_amd import shard  # noqa: E402
from openr_amd import topology as T  # noqa: E402
from openr_amd.engine import Engine  # noqa: E402
from openr_amd.linkstate import LinkState  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pods", type=int, default=1781)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--check", type=int, default=64)
    ap.add_argument("--no-digest", action="store_true", help="diagnostic: no digests")
    ap.add_argument("--no-dist", action="store_true", help="diagnostic: no u32 dist rows")
    args = ap.parse_args()
    st = T.fabric(pods=args.pods, planes=8)
    ls = LinkState(stream=st)
    csr = ls.csr()
    eng = Engine()
    eng.load(csr)
    V = eng.V
    dev = torch.device("cuda", 0)
    perm = np.random.default_rng(0x5EED).permutation(V).astype(np.uint32)
    nbrs = shard.distinct_neighbors(csr["row_ptr"], csr["col"])
    key = shard.first_neighbor(csr["row_ptr"], csr["col"])
    classes = shard.make_classes(perm, shard.neighbor_caps(nbrs), V,
                                 shard.last_neighbor(csr["row_ptr"], csr["col"]))
    order = np.concatenate([c.roots for c in classes])  # phase 1 order: class by class
    pos = np.empty(V, np.uint32)
    pos[order] = np.arange(V, dtype=np.uint32)
    d_order = torch.from_numpy(order.view(np.int32)).to(dev)
    d_pos = torch.from_numpy(pos.view(np.int32)).to(dev)
    lev = torch.empty((V, eng.lev_pitch), dtype=torch.uint8, device=dev)
    dist = torch.empty((V, V), dtype=torch.int32, device=dev)
    ldg = torch.empty((V, 3), dtype=torch.int64, device=dev)
    bufs = []
    for c in classes:
        bufs.append(dict(c=c, d=torch.from_numpy(c.roots.view(np.int32)).to(dev),
                         nh=torch.empty((c.roots.size, V, c.nh_words), dtype=torch.int32, device=dev),
                         dg=torch.empty((c.roots.size, 3), dtype=torch.int64, device=dev)))
    s = torch.cuda.current_stream()
    res = {"V": V, "phase1_ms": [], "phase2_ms": {}}
    for rep in range(args.reps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        eng.levels_dev(d_order.data_ptr(), V, lev.data_ptr(),
                       d_dist=0 if args.no_dist else dist.data_ptr(),
                       d_lev_digest=0 if args.no_digest else ldg.data_ptr(), stream=s.cuda_stream)
        e1.record(s)
        evs = []
        for b in bufs:
            a_, b_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a_.record(s)
            eng.nh_derive_dev(b["d"].data_ptr(), b["c"].roots.size, b["c"].nh_words, lev.data_ptr(),
                              d_pos.data_ptr(), b["nh"].data_ptr(),
                              d_lev_digest=0 if args.no_digest else ldg.data_ptr(),
                              d_digest=0 if args.no_digest else b["dg"].data_ptr(),
                              max_root_neighbors=b["c"].cap,
                              stream=s.cuda_stream)
            b_.record(s)
            evs.append((b["c"].cap, a_, b_))
        eng.sync(s.cuda_stream)
        if rep == 0:
            continue
        res["phase1_ms"].append(e0.elapsed_time(e1))
        for cap, a_, b_ in evs:
            res["phase2_ms"].setdefault(str(cap), []).append(a_.elapsed_time(b_))
        print(json.dumps({"rep": rep, "phase1_ms": res["phase1_ms"][-1],
                          "phase2_ms": {k: v[-1] for k, v in res["phase2_ms"].items()}}),
              file=sys.stderr, flush=True)
    # check sampled roots of every class against the per-batch engine path
    ok = True
    for b in (bufs if args.check > 0 else []):
        c = b["c"]
        idx = np.random.default_rng(1).choice(c.roots.size, min(args.check, c.roots.size),
                                              replace=False)
        roots = c.roots[idx]
        ref = eng.run(roots, c.nh_words, want_digest=True)
        dist_h = dist[torch.from_numpy(pos[roots].astype(np.int64)).to(dev)].cpu().numpy().view(np.uint32)
        nh_h = b["nh"][torch.from_numpy(idx.astype(np.int64)).to(dev)].cpu().numpy().view(np.uint32)
        dg_h = b["dg"][torch.from_numpy(idx.astype(np.int64)).to(dev)].cpu().numpy().view(np.uint64)
        ok &= bool(np.array_equal(dist_h, ref["dist"]) and np.array_equal(nh_h, ref["nh"]) and
                   np.array_equal(dg_h, ref["digest"]))
    res["check_equal"] = ok
    p1 = float(np.median(res["phase1_ms"]))
    p2 = {k: float(np.median(v)) for k, v in res["phase2_ms"].items()}
    res["median_phase1_ms"] = p1
    res["median_phase2_ms"] = p2
    res["step_ms"] = p1 + sum(p2.values())
    res["spf_per_s"] = V / (res["step_ms"] / 1e3)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
