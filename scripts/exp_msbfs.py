#!/usr/bin/env python3
"""Time the unit-metric classes (variant 5) of a topology's all-sources
sweep alone, one stream, under output-flag combinations and engine env
configs: how much of a class launch is the traversal, the rows, the digest."""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from openr_amd import _native as N  # noqa: E402
from openr_amd import shard  # noqa: E402
from openr_amd.engine import Engine  # noqa: E402
from openr_amd.linkstate import LinkState  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--topology", default="fabric100k")
ap.add_argument("--caps", type=int, nargs="+", default=[8, 96, 1792])
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--flags", nargs="+", default=["dist,nh,digest", "dist,nh", "dist", "digest"])
ap.add_argument("--envs", nargs="+", default=[""])
args = ap.parse_args()
torch.cuda.set_device(0)
st, desc, weighted, _ = bench.build_topology(args.topology)
ls = LinkState(stream=st)
csr = ls.csr()
eng = Engine(0)
eng.load(csr)
V = eng.V
nbrs = shard.distinct_neighbors(csr["row_ptr"], csr["col"])
caps = shard.neighbor_caps(nbrs)
perm = np.random.default_rng(bench.SEED).permutation(V).astype(np.uint32)
key = shard.first_neighbor(csr["row_ptr"], csr["col"])
classes = {c.cap: c for c in shard.make_classes(perm, caps, V, key, max_grouped_words=1)}
FL = {"dist": N.OSPF_WANT_DIST, "nh": N.OSPF_WANT_NH, "digest": N.OSPF_WANT_DIGEST}
s = torch.cuda.current_stream()
for cap in args.caps:
    c = classes[cap]
    n, W = c.roots.size, c.nh_words
    roots = torch.from_numpy(c.roots.astype(np.int32)).cuda()
    dist = torch.empty((n, V), dtype=torch.int32, device="cuda")
    nh = torch.empty((n, V, W), dtype=torch.int32, device="cuda")
    dig = torch.empty((n, 3), dtype=torch.int64, device="cuda")
    hint = int(nbrs[c.roots].max())
    for envc in args.envs:
        kv = [x.split("=") for x in envc.split(",") if x]
        for k_, v_ in kv:
            os.environ[k_] = v_
        for fl in args.flags:
            f = sum(FL[x] for x in fl.split(","))
            ts = []
            for r in range(args.reps + 1):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(s)
                eng.run_dev(roots.data_ptr(), n, W, flags=f, d_dist=dist.data_ptr(),
                            d_nh=nh.data_ptr(), d_digest=dig.data_ptr(), stream=s.cuda_stream,
                            max_root_neighbors=hint)
                b.record(s)
                b.synchronize()
                if r:
                    ts.append(a.elapsed_time(b))
            eng.sync(s.cuda_stream)
            ms = float(np.median(ts))
            print(json.dumps(dict(cap=cap, n=n, flags=fl, env=envc, ms=round(ms, 3),
                                  spf_s=round(n / ms * 1e3, 1))), flush=True)
        for k_, _ in kv:
            os.environ.pop(k_, None)
