#!/usr/bin/env python3
"""Time one width class of a topology's root sample in isolation (one stream,
back-to-back launches, HIP events) under several engine env configs.
Experiment harness for the weighted path (variant 7 knobs). One JSON line
per (class, config)."""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402  (topology table)
from openr_amd import _native as N  # noqa: E402
from openr_amd import shard  # noqa: E402
from openr_amd.engine import Engine  # noqa: E402
from openr_amd.linkstate import LinkState  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--topology", default="fabric100k-w")
ap.add_argument("--roots", type=int, default=4096)
ap.add_argument("--caps", type=int, nargs="+", default=[8, 16, 32, 96, 1792],
                help="neighbour-capacity classes (shard.neighbor_caps)")
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--envs", nargs="+", default=[""], help="'K=V,K=V' configs ('' = defaults)")
args = ap.parse_args()

torch.cuda.set_device(0)
st, desc, weighted, _ = bench.build_topology(args.topology)
ls = LinkState(stream=st)
csr = ls.csr()
eng = Engine(0)
eng.load(csr)
V, E = eng.V, csr["col"].size
nbrs = shard.distinct_neighbors(csr["row_ptr"], csr["col"])
caps = shard.neighbor_caps(nbrs)
perm = np.random.default_rng(bench.SEED).permutation(V).astype(np.uint32)[: args.roots]
flags = N.OSPF_WANT_DIST | N.OSPF_WANT_NH | N.OSPF_WANT_DIGEST
s = torch.cuda.current_stream()
for cap in args.caps:
    members = perm[caps[perm] == cap]
    W = max(1, (cap + 31) // 32)
    n = members.size
    if n == 0:
        continue
    roots = torch.from_numpy(members.astype(np.int32)).cuda()
    dist = torch.empty((n, V), dtype=torch.int32, device="cuda")
    nh = torch.empty((n, V, W), dtype=torch.int32, device="cuda")
    dig = torch.empty((n, 3), dtype=torch.int64, device="cuda")
    hint = int(nbrs[members].max())
    ref = None
    for envc in args.envs:
        kv = [x.split("=") for x in envc.split(",") if x]
        for k_, v_ in kv:
            os.environ[k_] = v_
        ts = []
        for r in range(args.reps + 1):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            eng.run_dev(roots.data_ptr(), n, W, flags=flags, d_dist=dist.data_ptr(),
                        d_nh=nh.data_ptr(), d_digest=dig.data_ptr(), stream=s.cuda_stream,
                        max_root_neighbors=hint)
            b.record(s)
            b.synchronize()
            if r:
                ts.append(a.elapsed_time(b))
        eng.sync(s.cuda_stream)
        got = dig.cpu().numpy().copy()
        same = None if ref is None else bool(np.array_equal(got, ref))
        ref = got if ref is None else ref
        for k_, _ in kv:
            os.environ.pop(k_, None)
        ms = float(np.median(ts))
        print(json.dumps(dict(topology=args.topology, cap=cap, W=W, n=n, env=envc, ms=round(ms, 3),
                              spf_s=round(n / ms * 1e3, 1), same_digests=same)), flush=True)
