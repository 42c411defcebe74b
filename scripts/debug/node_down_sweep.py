#!/usr/bin/env python3
"""Round 6 diagnosis: prod_callstack's [NODE DOWN] all-sources re-sweep
stalled (F100k with one rack deleted: V = 100,023, not a multiple of 4).
Runs that sweep on a fabric of --pods pods after one rack's database is
deleted, with the sweep's host phases on stderr and the Python stack dumped
every 20 s, and checks the digests of a few roots against the oracle."""
import argparse
import faulthandler
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ.setdefault("OSPF_SWEEP_TIMING", "1")

import torch  # noqa: E402,F401

from openr_amd import topology as T  # noqa: E402
from openr_amd.adjdb import AdjDb, AdjDbStream  # noqa: E402
from openr_amd.linkstate import LinkState  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--pods", type=int, default=64)
ap.add_argument("--delete", default="3-2-7")
args = ap.parse_args()
faulthandler.dump_traceback_later(20, repeat=True)
st = T.fabric(pods=args.pods, planes=8)
p = LinkState()
p.apply(st)
t = time.perf_counter()
p.prefetch_all()
print(f"pods={args.pods} V={p.num_nodes()} sweep {1e3 * (time.perf_counter() - t):.1f} ms", flush=True)
p.apply(AdjDbStream.from_dbs([AdjDb(args.delete, delete=True)]))
p.prefetch(["3-0-0"])
print(f"after delete V={p.num_nodes()}", flush=True)
t = time.perf_counter()
p.prefetch_all()
print(f"sweep after delete {1e3 * (time.perf_counter() - t):.1f} ms", flush=True)
d = p.all_sources_digests()
names = p.node_names()
from oracle import Oracle  # noqa: E402  (checker)
o = Oracle(AdjDbStream.from_dbs([x for x in st.to_dbs() if x.name != args.delete]))
bad = 0
for i in list(range(0, len(names), max(1, len(names) // 40))):
    od = o.digests([names[i]])
    bad += int(not (od[0] == d[i]).all())
print(f"digest mismatches {bad}", flush=True)
faulthandler.cancel_dump_traceback_later()
sys.exit(1 if bad else 0)
