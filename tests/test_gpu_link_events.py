"""[LINK UP] / [LINK DOWN] patched in place (SURVEY §8
f4): an adjacency database that adds or withdraws links between known nodes
(LinkState::updateAdjacencyDatabase, openr/decision/LinkState.cpp:632-657;
Decision applies one database per KvStore key, Decision.cpp:743-765) patches
odl::LinkState's CSR and the device graph in place (ospf_update_rows) -- no
whole snapshot, no device reload -- and every result after every event equals
the CPU oracle's: full SpfResult text (metric, next hops, ordered pathLinks)
of link-metric and hop-count runs, KSP2 paths, all-sources sweep digests,
decision.spf_runs."""
import numpy as np
import pytest

import link_events as LE
from graphs import drained_fabric
from link_events import apply_both, both, withdraw
from oracle import Oracle  # noqa: F401
from openr_amd import topology as T
from openr_amd.adjdb import AdjDb, AdjDbStream, create_adjacency
from openr_amd.engine import Engine
from openr_amd.linkstate import LinkState

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed", range(4))
@pytest.mark.parametrize("unit", [False, True])
def test_link_down_up_random_graphs(seed, unit):
    LE.link_down_up_random_graphs(seed, unit)


def test_link_events_mixed_with_metric_and_overload():
    LE.link_events_mixed_with_metric_and_overload()


def test_parallel_link_ranks_after_insert():
    LE.parallel_link_ranks_after_insert()


def test_engine_update_rows_equals_fresh_load():
    """Engine level: ospf_update_rows after links removed and added equals a
    fresh ospf_load_graph of the same CSR -- dist, next-hop rows and digests
    of every root -- including rows that outgrow their padded slots (a rack
    of a fabric gains links: every later row moves) and the layout reserve
    running out (OSPF_E_RANGE, then a reload)."""
    st = T.fabric(pods=6, planes=4)
    ls = LinkState()
    ls.apply(st)
    names = ls.node_names()
    V = len(names)
    eng = Engine()
    eng.load(ls.csr())
    dbs = {d.name: d for d in st.to_dbs()}
    rng = np.random.default_rng(0)
    version = 2
    for step in range(12):
        ids0 = ls.node_names()
        if step % 2 == 0:  # a new link rack - rack (rows of 4 + 0 -> slots grow)
            a, b = rng.choice([n for n in names if n.startswith("3-")], 2, replace=False).tolist()
            dbs[a].adjs.append(create_adjacency(b, f"{a}-{b}-e{step}", f"{b}-{a}-e{step}", 1))
            dbs[b].adjs.append(create_adjacency(a, f"{b}-{a}-e{step}", f"{a}-{b}-e{step}", 1))
            ls.apply(AdjDbStream.from_dbs([dbs[a], dbs[b]]))
            rows = [ids0.index(a), ids0.index(b)]
        else:  # a link withdrawn
            a = rng.choice(names).item()
            if not dbs[a].adjs:
                continue
            adj = dbs[a].adjs.pop(int(rng.integers(len(dbs[a].adjs))))
            ls.apply(AdjDbStream.from_dbs([dbs[a]]))
            rows = [ids0.index(a), ids0.index(adj.other)]
        csr = ls.csr()
        eng.update_rows(csr, rows, version)
        version += 1
        fresh = Engine()
        fresh.load(csr)
        W = max(fresh.nh_words(r) for r in range(V))
        all_ = np.arange(V, dtype=np.uint32)
        got = eng.run(all_, W, want_digest=True)
        want = fresh.run(all_, W, want_digest=True)
        for k in ("dist", "nh", "digest"):
            assert np.array_equal(got[k], want[k]), (step, k)
        assert eng.info().n_edges == fresh.info().n_edges
        fresh.close()
    eng.close()


@pytest.mark.timeout(600)
def test_f10k_link_down_up_sweep_in_place():
    """A drained F10k: a rack's uplink withdrawn and restored, a spine link
    withdrawn, a new rack - rack link; the all-sources sweep digests after
    each event equal the CSR-Dijkstra restatement's for every root, with no
    snapshot and no device load after the first."""
    st = drained_fabric(173, 8, seed=4, drain=0.01, down=0.005)
    o, p = both(st)
    names = p.node_names()
    dbs = {d.name: d for d in st.to_dbs()}
    p.prefetch_all()
    s0 = p.topology_stats()
    evs = []
    rack, spine = "3-17-5", "1-2-7"
    db, adj = withdraw(dbs, rack, 0)
    evs.append([db])
    evs.append("restore")
    db2, adj2 = withdraw(dbs, spine, 3)
    evs.append([db2])
    for ev in evs:
        if ev == "restore":
            dbs[rack].adjs.insert(0, adj)
            ev = [dbs[rack]]
        apply_both(o, p, ev)
        got = p.all_sources_digests()
        assert np.array_equal(got, o.fast_digests(names, True, threads=16))
        for r in (rack, spine, "2-17-3"):
            assert p.spf_text(r) == o.spf_text(r), r
    s1 = p.topology_stats()
    assert s1["snapshots"] == s0["snapshots"] and s1["loads"] == s0["loads"], (s0, s1)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("pods", [64, 173])
def test_fabric_node_down_up_sweep(pods):
    """[NODE DOWN] / [NODE UP] of a rack on a fabric: the node count leaves
    the multiples of 4 (unaligned row pitches in the derive sweep: round 6's
    prod_callstack found its twin next-hop launch refusing them) and comes
    back; the all-sources digests after each event equal the CSR-Dijkstra
    restatement's for every root, on the engine (ODL_STRICT_ENGINE: no host
    fallback)."""
    st = drained_fabric(pods, 8, seed=5, drain=0.01, down=0.005)
    o, p = both(st)
    p.prefetch_all()
    dbs = {d.name: d for d in st.to_dbs()}
    rack = "3-7-5"
    for ev in ([AdjDb(rack, delete=True)], [dbs[rack]]):
        apply_both(o, p, ev)
        names = p.node_names()
        assert p.all_sources_digests().tolist() == o.fast_digests(names, True, threads=16).tolist()
        assert p.spf_text("3-0-0") == o.spf_text("3-0-0")
    assert p.sweep_stats()["mode"] == "derive"
    assert not p.counters()["engine_degraded"]


@pytest.mark.parametrize("seed", range(2))
@pytest.mark.parametrize("unit", [False, True])
def test_node_remove_add_in_place(seed, unit):
    """Nodes withdrawn, restored and added in place on the host snapshot; the
    engine reloads the renumbered graph (one device load per event), results
    == the oracle after every event."""
    s0, s1 = LE.node_remove_add_random_graphs(seed, unit)
    assert s1["loads"] > s0["loads"]
