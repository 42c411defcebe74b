#!/usr/bin/env python3
"""Round 6 diagnosis: what the first getSpfResult-shaped run on a freshly
loaded F100k graph pays beyond a warm one, in a fresh process (no torch CUDA
init): ospf_open, ospf_load_graph (twice: first touch vs reuse), then
single-root batches (dist + next hops) for a rack, a fabric switch and a
spine, each twice. Prints one JSON line of wall-clock ms."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from openr_amd import topology as T  # noqa: E402
from openr_amd.engine import Engine  # noqa: E402
from openr_amd.linkstate import LinkState  # noqa: E402

out = {}
st = T.fabric(pods=1781, planes=8)
ls = LinkState()
ls.set_host_spf(True)
ls.apply(st)
csr = ls.csr()
names = ls.node_names()
ids = {n: i for i, n in enumerate(names)}


def ms(f):
    t = time.perf_counter()
    r = f()
    return r, round((time.perf_counter() - t) * 1e3, 3)


eng, out["open_ms"] = ms(Engine)
_, out["load1_ms"] = ms(lambda: eng.load(csr, 1))
_, out["load2_ms"] = ms(lambda: eng.load(csr, 2))
for name in ("3-0-0", "2-5-3", "1-2-7"):
    r = ids[name]
    W = eng.nh_words(r)
    _, a = ms(lambda: eng.run([r], W))
    _, b = ms(lambda: eng.run([r], W))
    out[f"run_{name}_first_ms"], out[f"run_{name}_second_ms"] = a, b
print(json.dumps(out), flush=True)
