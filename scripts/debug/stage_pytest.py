#!/usr/bin/env python3
"""Debug: the failing test_twin_levels_forced_and_off[1] sequence in one
process (seed 0 then seed 1), printing row diffs of mismatching roots."""
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


def check(eng, names, tag):
    V = eng.V
    sw = Sweep(eng, mode="derive")
    sw.run()
    eng.sync()
    d = np.zeros((V, 3), np.uint64)
    sw._check(sw._L.ospf_sweep_digests_host(sw._h, d.ctypes.data))
    got = dict(zip(sw.roots.tolist(), d))
    words = np.array([eng.nh_words(r) for r in range(V)])
    bad = []
    for W in sorted(set(words.tolist())):
        grp = np.nonzero(words == W)[0].astype(np.uint32)
        ref = eng.run(grp, W, want_digest=True)
        for j, r in enumerate(grp.tolist()):
            if not np.array_equal(got[r], ref["digest"][j]):
                bad.append((r, W, ref["dist"][j]))
    print(tag, "mismatches", len(bad), [names[b[0]] for b in bad[:10]], flush=True)
    for r, W, rd in bad[:3]:
        dist, nh = sw.rows(np.array([r], np.uint32), W)
        dd = np.nonzero(dist[0] != rd)[0]
        print("   ", names[r], "dist diffs", dd.size, [names[x] for x in dd[:6]], dist[0][dd[:6]].tolist(),
              rd[dd[:6]].tolist(), flush=True)
    print("    units", [(p["name"], p["n_roots"]) for p in sw.profile(1)], flush=True)
    sw.close()


for seed in (0, 1):
    os.environ["OSPF_SWEEP_STAGES"] = "1" if seed == 0 else "8"
    st = drained_fabric(7, 4, seed=seed + 3, drain=0.07, down=0.05)
    for env in ("OSPF_SWEEP_TWINLV", "OSPF_SWEEP_NOTWINLV"):
        os.environ[env] = "1"
        ls = LinkState()
        ls.apply(st)
        eng = Engine()
        eng.load(ls.csr())
        check(eng, ls.node_names(), f"seed={seed} {env}")
        eng.close()
        del os.environ[env]
