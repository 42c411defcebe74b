#!/usr/bin/env python3
"""Debug: derive-sweep digests vs the batch path on a drained fabric under
forced twin levels and pipeline stages, eager and graph-replayed."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: F401,E402

from graphs import drained_fabric  # noqa: E402
from openr_amd.engine import Engine, Sweep  # noqa: E402
from openr_amd.linkstate import LinkState  # noqa: E402

os.environ["OSPF_SWEEP_TWINLV"] = "1"
# dirty device memory first (pytest runs other GPU tests before): freed
# allocations come back holding old bytes
junk = torch.full((1 << 30,), 0x5A, dtype=torch.uint8, device="cuda")
del junk
torch.cuda.empty_cache()
for stages in ("1", "8"):
    os.environ["OSPF_SWEEP_STAGES"] = stages
    st = drained_fabric(7, 4, seed=4, drain=0.07, down=0.05)
    ls = LinkState()
    ls.apply(st)
    csr = ls.csr()
    names = ls.node_names()
    eng = Engine()
    eng.load(csr)
    V = eng.V
    words = np.array([eng.nh_words(r) for r in range(V)])
    ref = {}
    for W in sorted(set(words.tolist())):
        grp = np.nonzero(words == W)[0].astype(np.uint32)
        out = eng.run(grp, W, want_digest=True)
        for j, r in enumerate(grp.tolist()):
            ref[r] = out["digest"][j]
    for hg in (False, True):
        sw = Sweep(eng, mode="derive", hip_graph=hg)
        sw.run()
        eng.sync()
        d = np.zeros((V, 3), np.uint64)
        sw._check(sw._L.ospf_sweep_digests_host(sw._h, d.ctypes.data))
        got = dict(zip(sw.roots.tolist(), d))
        bad = [r for r in range(V) if not np.array_equal(got[r], ref[r])]
        names_bad = [names[r] for r in bad]
        print(f"stages={stages} graph={hg} mismatches={len(bad)} {names_bad[:12]}", flush=True)
        for r in bad[:4]:
            print("   ", names[r], got[r].tolist(), ref[r].tolist(), flush=True)
        if bad:
            ls2 = LinkState()
            ls2.apply(st)
            dist, nh = sw.rows(np.array(bad[:2], np.uint32), 1)
            refr = eng.run(np.array(bad[:2], np.uint32), 1)
            for i, r in enumerate(bad[:2]):
                dd = np.nonzero(dist[i] != refr["dist"][i])[0]
                print("    dist diff", names[r], dd.size, dist[i][dd[:8]].tolist(), refr["dist"][i][dd[:8]].tolist())
        print("   units:", [p["name"] for p in sw.profile(1)], flush=True)
        sw.close()
    eng.close()
