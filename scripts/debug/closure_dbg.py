"""Closure split / plan decision on the closure test fabric (stderr lines of
OSPF_SWEEP_DEBUG), and the sweep's units."""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
os.environ["OSPF_SWEEP_DEBUG"] = "1"
from graphs import drained_fabric  # noqa: E402
from openr_amd.engine import Engine, Sweep  # noqa: E402
from openr_amd.linkstate import LinkState  # noqa: E402

st = drained_fabric(40, 4, seed=5, drain=0.0, down=0.0, weighted_seed=11, ssw_per_plane=4)
ls = LinkState()
ls.apply(st)
eng = Engine()
eng.load(ls.csr())
sw = Sweep(eng, mode="wcover")
print([p["name"] for p in sw.profile(1)], flush=True)
sw.close()
eng.close()
