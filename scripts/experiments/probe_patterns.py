"""Store-pattern sweep with ospf_probe_store: which row-block shapes reach the
streaming store rate (leaf launch layout: 2 x [rows][V] u32)."""
import json, sys, os
import numpy as np
import torch  # noqa: F401
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from openr_amd.engine import Engine
V, rows = 100024, 83707
e = Engine(0)
out = []
def run(p, g, ct):
    ms = float(np.median(e.probe_store(p, V, rows, g, ct, reps=3)))
    r = {"pattern": p, "group": g, "ctiles": ct, "ms": round(ms, 3),
         "GBs": round(2 * rows * V * 4 / ms / 1e6, 1)}
    print(json.dumps(r), flush=True)
    out.append(r)
pats = sys.argv[1].split(",") if len(sys.argv) > 1 else ["rows_chunk", "rows_group"]
groups = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1, 2, 4, 8, 16, 48, 64]
cts = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [1, 2, 6, 20, 98]
run("stream", 48, 6)
for g in groups:
    for ct in cts:
        for p in pats:
            run(p, g, ct)
run("stream", 48, 6)
