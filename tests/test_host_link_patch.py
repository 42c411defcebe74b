"""CPU: the in-place structural patch of odl::LinkState's CSR snapshot
(links added / removed between known nodes, LinkState.cpp:632-657) equals a
whole re-snapshot of the same live link sets after every event -- rows,
neighbour order, link ranks (linksFromNode iteration order), metrics, up
bits, twins and the link behind every entry. The reference LinkState is the
model: the patched snapshot must describe exactly the graph a fresh one
would."""
import os

import numpy as np
import pytest

from graphs import random_stream
from openr_amd.adjdb import AdjDb, AdjDbStream, create_adjacency
from openr_amd.linkstate import LinkState


def csr_view(ls):
    c = ls.csr()
    keys = ls.link_keys()
    c["key"] = np.array([keys[i] for i in c["link_id"]], dtype=object)
    return c


def same(a, b):
    for k in ("row_ptr", "col", "metric", "edge_up", "link_rank", "no_transit", "twin", "key"):
        assert np.array_equal(a[k], b[k]), k


def apply(ls, dbs, patch):
    if patch:
        os.environ.pop("ODL_NO_LINK_PATCH", None)
    else:
        os.environ["ODL_NO_LINK_PATCH"] = "1"
    try:
        return ls.apply(AdjDbStream.from_dbs(dbs))
    finally:
        os.environ.pop("ODL_NO_LINK_PATCH", None)


@pytest.mark.parametrize("seed", range(6))
def test_patched_snapshot_equals_resnapshot(seed):
    st, names = random_stream(400 + seed, n=30, p=0.2, parallel=0.3)
    p, q = LinkState(), LinkState()
    p.apply(st)
    q.apply(st)
    same(csr_view(p), csr_view(q))
    s0 = p.topology_stats()
    rng = np.random.default_rng(seed)
    dbs = {d.name: d for d in st.to_dbs()}
    for step in range(40):
        a = names[int(rng.integers(len(names)))]
        kind = int(rng.integers(3))
        if kind == 0 and dbs[a].adjs:  # withdraw (+ metric / overload changes of others)
            dbs[a].adjs.pop(int(rng.integers(len(dbs[a].adjs))))
            if len(dbs[a].adjs) > 1 and rng.random() < 0.5:
                dbs[a].adjs[0].overloaded = not dbs[a].adjs[0].overloaded
                dbs[a].adjs[1].metric = int(rng.integers(1, 30))
            ups = [dbs[a]]
        else:  # add a link (maybe parallel to one that exists)
            b = names[int(rng.integers(len(names)))]
            if b == a:
                continue
            ia, ib = f"{a}-{b}-p{step}", f"{b}-{a}-p{step}"
            dbs[a].adjs.append(create_adjacency(b, ia, ib, int(rng.integers(1, 30)),
                                                overloaded=bool(rng.random() < 0.2)))
            dbs[b].adjs.append(create_adjacency(a, ib, ia, int(rng.integers(1, 30))))
            ups = [dbs[a], dbs[b]]
        ca = apply(p, ups, True)
        cb = apply(q, ups, False)
        assert ca == cb
        same(csr_view(p), csr_view(q))
    s1 = p.topology_stats()
    assert s1["snapshots"] == s0["snapshots"], (s0, s1)
    assert s1["link_patches"] > s0["link_patches"]
    # q took a snapshot per structural event
    assert q.topology_stats()["link_patches"] == 0


def test_rank_change_on_rehash_is_followed():
    """A hub whose LinkSet rehashes as links are added: ranks of its other
    links move; the patched rows follow them."""
    adj = {f"h{i}": [] for i in range(6)}
    dbs = {nm: AdjDb(nm, adj[nm], i + 1) for i, nm in enumerate(adj)}
    for i in range(1, 6):
        for k in range(2):
            a, b = "h0", f"h{i}"
            dbs[a].adjs.append(create_adjacency(b, f"{a}-{b}-{k}", f"{b}-{a}-{k}", 2))
            dbs[b].adjs.append(create_adjacency(a, f"{b}-{a}-{k}", f"{a}-{b}-{k}", 2))
    st = AdjDbStream.from_dbs(list(dbs.values()))
    p, q = LinkState(), LinkState()
    p.apply(st)
    q.apply(st)
    for step in range(60):
        b = f"h{1 + step % 5}"
        ia, ib = f"h0-{b}-x{step}", f"{b}-h0-x{step}"
        dbs["h0"].adjs.append(create_adjacency(b, ia, ib, 2))
        dbs[b].adjs.append(create_adjacency("h0", ib, ia, 2))
        apply(p, [dbs["h0"], dbs[b]], True)
        apply(q, [dbs["h0"], dbs[b]], False)
        same(csr_view(p), csr_view(q))
