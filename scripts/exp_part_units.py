#!/usr/bin/env python3
"""Round 6 diagnosis: per-launch-unit times (ospf_sweep_profile) of the F100k
sweep alone and of part 0 of 2 / 4 / 8 root-partition parts, to see which
units keep a part from taking 1/N of the single sweep. One JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402,F401

from openr_amd import topology as T  # noqa: E402
from openr_amd.engine import Engine, Sweep  # noqa: E402
from openr_amd.linkstate import LinkState  # noqa: E402

ls = LinkState()
ls.set_host_spf(True)
ls.apply(T.fabric(pods=1781, planes=8))
eng = Engine()
eng.load(ls.csr())
out = {}
variants = [("", None)] + [(v, v.split("=")) for v in sys.argv[1:]]
for tag, kv in variants:
    if kv:
        os.environ[kv[0]] = kv[1]
    for n in (1, 2, 4, 8):
        sw = Sweep(eng, part=0, n_parts=n)
        sw.run()
        eng.sync()
        units = sw.profile(3)
        out[f"{tag or 'base'}/{n}"] = {"roots": sw.n_roots, "rows": sw.n_rows,
                                       "sum_ms": round(sum(u["ms_median"] for u in units), 3),
                                       "units": {u["name"]: [u["n_roots"], round(u["ms_median"], 3)] for u in units}}
        sw.close()
    if kv:
        os.environ.pop(kv[0])
print(json.dumps(out), flush=True)
