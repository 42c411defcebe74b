"""Row-pitch alignment A/B with ospf_probe_store: the leaf launch's rows at
V = 100,024 (a 400,096-B pitch: rows 32-B but not 128-B aligned) vs the
pitch padded to 64 nodes (256-B aligned rows)."""
import json, sys, os
import numpy as np
import torch  # noqa: F401
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from openr_amd.engine import Engine
rows = 83707
e = Engine(0)
for rep in range(2):
    for V in (100024, 100032, 100064, 100096, 100028):
        for p, g, ct in (("stream", 48, 6), ("rows_chunk", 48, 6), ("rows_chunk", 8, 6), ("rows_walk", 1, 8)):
            ms = float(np.median(e.probe_store(p, V, rows, g, ct, reps=3)))
            print(json.dumps({"V": V, "pitch_mod_256": (V * 4) % 256, "pattern": p, "group": g,
                              "ctiles": ct, "ms": round(ms, 3),
                              "GBs": round(2 * rows * V * 4 / ms / 1e6, 1)}), flush=True)
