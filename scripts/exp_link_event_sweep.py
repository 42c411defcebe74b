#!/usr/bin/env python3
"""Round 6 A/B, one process: the all-sources re-sweep after [LINK DOWN] /
[LINK UP] at F100k (odl::LinkState::prefetchAllSources: plan + first run)
with the first run's serial prefix started while the plan is built
(OSPF_SWEEP_EARLY_START, the default) and without it (OSPF_SWEEP_NO_EARLY,
read at each sweep's create). Each event's digests are compared across the
two modes. Prints one JSON line."""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from openr_amd import topology as T  # noqa: E402
from openr_amd.adjdb import AdjDbStream  # noqa: E402
from openr_amd.linkstate import LinkState  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
st = T.fabric(pods=1781, planes=8)
p = LinkState()
p.apply(st)
p.prefetch_all()
db = [d for d in st.to_dbs() if d.name == "3-901-0"][0]
adj = db.adjs[0]
times = {"early": {"down": [], "up": []}, "no_early": {"down": [], "up": []}}
dig = {}
for i in range(reps):
    mode = "early" if i % 2 == 0 else "no_early"
    if mode == "no_early":
        os.environ["OSPF_SWEEP_NO_EARLY"] = "1"
    else:
        os.environ.pop("OSPF_SWEEP_NO_EARLY", None)
    for kind in ("down", "up"):
        if kind == "down":
            db.adjs.remove(adj)
        else:
            db.adjs.insert(0, adj)
        p.apply(AdjDbStream.from_dbs([db]))
        t = time.perf_counter()
        p.prefetch_all()
        times[mode][kind].append((time.perf_counter() - t) * 1e3)
        d = p.all_sources_digests()
        if kind in dig:
            assert np.array_equal(dig[kind], d), (mode, kind)
        dig[kind] = d
    print(mode, {k: round(v[-1], 2) for k, v in times[mode].items()}, file=sys.stderr, flush=True)
out = {m: {k: {"median_ms": round(statistics.median(v), 2), "ms": [round(x, 2) for x in v]}
           for k, v in kv.items()} for m, kv in times.items()}
out["digests_equal_across_modes"] = True
print(json.dumps(out), flush=True)
