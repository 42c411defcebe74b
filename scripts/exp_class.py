#!/usr/bin/env python3
"""Time one root class of the F100k all-sources sweep in isolation (one
stream, back-to-back launches, HIP events). Experiment harness for kernel
knobs (OSPF_BLOCK, OSPF_FORCE_VARIANT). Prints one JSON line per config."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openr_amd import _native as N  # noqa: E402
from openr_amd import shard, topology as T  # noqa: E402
from openr_amd.engine import Engine  # noqa: E402
from openr_amd.linkstate import LinkState  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--pods", type=int, default=1781)
ap.add_argument("--planes", type=int, default=8)
ap.add_argument("--W", type=int, nargs="+", default=[1, 3, 56])
ap.add_argument("--n", type=int, nargs="+", default=[256, 1024, 4096])
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--blocks", type=int, nargs="+", default=[0])
ap.add_argument("--envs", nargs="+", default=[""],
                help="engine env configs to sweep, each 'K=V,K=V' ('' = defaults)")
ap.add_argument("--order", choices=["auto", "random", "locality"], default="auto",
                help="auto = locality for single-word classes (as bench.py)")
args = ap.parse_args()

torch.cuda.set_device(0)
st = T.fabric(pods=args.pods, planes=args.planes)
ls = LinkState(stream=st)
csr = ls.csr()
eng = Engine(0)
eng.load(csr)
V, E = eng.V, csr["col"].size
nbrs = shard.distinct_neighbors(csr["row_ptr"], csr["col"])
words = np.maximum(1, (nbrs + 31) // 32)
perm = np.random.default_rng(1).permutation(V).astype(np.uint32)
flags = N.OSPF_WANT_DIST | N.OSPF_WANT_NH | N.OSPF_WANT_DIGEST
s = torch.cuda.current_stream()
for W in args.W:
    members = perm[words[perm] == W]
    if args.order == "locality" or (args.order == "auto" and W == 1):
        members = shard.locality_order(members, shard.first_neighbor(csr["row_ptr"], csr["col"]))
    if members.size == 0:
        continue
    for n in args.n:
        roots = torch.from_numpy(np.resize(members, n).astype(np.int32)).cuda()
        dist = torch.empty((n, V), dtype=torch.int32, device="cuda")
        nh = torch.empty((n, V, W), dtype=torch.int32, device="cuda")
        dig = torch.empty((n, 3), dtype=torch.int64, device="cuda")
        for blk, envc in [(b_, e_) for b_ in args.blocks for e_ in args.envs]:
            for kv in [x for x in envc.split(",") if x]:
                k_, v_ = kv.split("=")
                os.environ[k_] = v_
            if blk:
                os.environ["OSPF_BLOCK"] = str(blk)
            else:
                os.environ.pop("OSPF_BLOCK", None)
            hint = int(nbrs[members].max())
            plan = eng.plan(W, flags, n_roots=n, max_root_neighbors=hint)
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
            for kv in [x for x in envc.split(",") if x]:
                os.environ.pop(kv.split("=")[0], None)
            ms = float(np.median(ts))
            print(json.dumps(dict(W=W, n=n, env=envc, order=args.order, pack=os.environ.get("OSPF_MS_PACK"), plan=plan, ms=round(ms, 3),
                                  spf_s=round(n / ms * 1e3, 1),
                                  us_per_root=round(ms * 1e3 / n, 2),
                                  gteps=round(n * E / ms / 1e6, 2))), flush=True)
