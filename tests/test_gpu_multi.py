"""Multi-GPU readiness on a one-GPU box:
the root partition at 2 / 4 / 8 parts reproduces the single sweep (every
root once, digests bit for bit), and the multi-device context's digest
gather through RCCL (one ncclAllGather of the parts' padded 24-B records;
here a one-rank communicator, OSPF_RCCL=1) equals the peer-copy gather and
the single sweep. Reference: Decision runs in one process on one thread
(openr/Main.cpp:515-527), so the drop-in reaches a node's GPUs from there."""
import numpy as np
import pytest

from graphs import drained_fabric
from openr_amd import topology as T
from openr_amd.engine import Engine, Multi, MultiSweep, Sweep
from openr_amd.linkstate import LinkState

pytestmark = pytest.mark.gpu


def sweep_digests(sw, V):
    d = np.zeros((max(1, sw.n_roots), 3), np.uint64)
    sw._check(sw._L.ospf_sweep_digests_host(sw._h, d.ctypes.data))
    out = np.zeros((V, 3), np.uint64)
    out[sw.roots] = d[: sw.n_roots]
    return out


@pytest.mark.parametrize("weighted", [False, True])
def test_parts_union_equals_single_sweep(weighted):
    st = drained_fabric(40, 8, seed=9, drain=0.02, down=0.01,
                        weighted_seed=7 if weighted else None)
    ls = LinkState()
    ls.apply(st)
    eng = Engine()
    eng.load(ls.csr())
    V = eng.V
    full = Sweep(eng)
    full.run()
    eng.sync()
    want = sweep_digests(full, V)
    full.close()
    for n in (2, 4, 8):
        got = np.zeros((V, 3), np.uint64)
        seen = np.zeros(V, np.int32)
        for i in range(n):
            p = Sweep(eng, part=i, n_parts=n)
            p.run()
            eng.sync()
            d = sweep_digests(p, V)
            seen[p.roots] += 1
            got[p.roots] = d[p.roots]
            p.close()
        assert np.all(seen == 1), n
        assert np.array_equal(got, want), n
    eng.close()


@pytest.mark.parametrize("rccl", ["1", "0"])
def test_multi_gather_rccl_one_rank(rccl, monkeypatch):
    monkeypatch.setenv("OSPF_RCCL", rccl)
    st = T.fabric(pods=12, planes=4)
    ls = LinkState()
    ls.apply(st)
    csr = ls.csr()
    eng = Engine()
    eng.load(csr)
    V = eng.V
    full = Sweep(eng)
    full.run()
    eng.sync()
    want = sweep_digests(full, V)
    full.close()
    eng.close()
    m = Multi([0])
    m.load(csr)
    ms = MultiSweep(m, hip_graph=False)
    assert ms.gather_backend == ("rccl" if rccl == "1" else "peer")
    ms.run()
    assert np.array_equal(ms.digests(), want)
    ms.run()  # a second gather through the same communicator
    assert np.array_equal(ms.digests(), want)
    ms.close()
    m.close()
