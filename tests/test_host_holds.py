"""Link hold TTLs (VERDICT r05 missing #3): HoldableValue semantics
(openr/decision/LinkState.cpp:48-117), Link::decrementHolds / hasHolds
(:237-263), LinkState::decrementHolds / hasHolds (:520-548) and the TTL
arguments of updateAdjacencyDatabase (:585-700), through odl::LinkState's
odl_apply_hold / odl_decrement_holds / odl_has_holds.

test_holdable_value_* transcribe LinkStateTest.cpp:22-83
(HoldableValueTest.BasicOperation): HoldableValue<bool> as a node's overload
bit (isNodeOverloaded), HoldableValue<LinkStateMetric> as a link's metric
from one end (linksFromNode). The SPF tests check that a held change is not
seen by SPF until its hold expires: getSpfResult text against the oracle
(CPU restatement) of the graph as it is in effect -- before the change while
held, after it once expired. Each runs GPU-free (odl_set_host_spf) and,
under -m gpu, on the engine."""
import numpy as np
import pytest

from oracle import Oracle
from openr_amd.adjdb import AdjDb, AdjDbStream, create_adjacency
from openr_amd.linkstate import LinkState

UP, DOWN = 10, 5  # holdUpTtl, holdDownTtl of LinkStateTest.cpp:27

MODE = {"spf": "host"}


@pytest.fixture(autouse=True, params=["host", pytest.param("gpu", marks=pytest.mark.gpu)])
def spf_mode(request):
    MODE["spf"] = request.param
    yield request.param
    MODE["spf"] = "host"


def _ls():
    p = LinkState()
    p.set_host_spf(MODE["spf"] == "host")
    return p


def _pair(m12=10, m21=10, ov1=False, ov2=False):
    a = AdjDb("1", [create_adjacency("2", "1/2", "2/1", m12)], 1, overloaded=ov1)
    b = AdjDb("2", [create_adjacency("1", "2/1", "1/2", m21)], 2, overloaded=ov2)
    return a, b


def _upd(p, db, up=UP, down=DOWN):
    return p.apply(AdjDbStream.from_dbs([db]), hold_up_ttl=up, hold_down_ttl=down)[0]


def test_holdable_value_bool_as_node_overload():
    p = _ls()
    a, b = _pair(ov1=True)
    p.apply(AdjDbStream.from_dbs([a, b]))
    assert p.is_overloaded("1") and not p.has_holds()
    assert not p.decrement_holds()
    # change bringing up (overload cleared): held UP calls
    a.overloaded = False
    assert not _upd(p, a)[0]
    for _ in range(UP - 1):
        assert p.has_holds() and p.is_overloaded("1")
        assert not p.decrement_holds()
    assert p.decrement_holds()  # expire the hold
    assert not p.has_holds() and not p.is_overloaded("1")
    # no hold since the value did not change
    assert not _upd(p, a)[0]
    assert not p.has_holds() and not p.is_overloaded("1")
    # change bringing down now: held DOWN calls
    a.overloaded = True
    assert not _upd(p, a)[0]
    for _ in range(DOWN - 1):
        assert p.has_holds() and not p.is_overloaded("1")
        assert not p.decrement_holds()
    assert p.decrement_holds()
    assert not p.has_holds() and p.is_overloaded("1")
    # change twice within the TTL: the second drops the hold (fast update)
    a.overloaded = False
    assert not _upd(p, a)[0]
    assert p.has_holds() and p.is_overloaded("1")
    assert not p.decrement_holds()
    a.overloaded = True
    assert _upd(p, a)[0]
    assert not p.has_holds() and p.is_overloaded("1")


def _metric(p, node):
    (_, m, _), = p.links(node)
    return m


def test_holdable_value_metric_as_link_metric():
    p = _ls()
    a, b = _pair()
    p.apply(AdjDbStream.from_dbs([a, b]))
    assert _metric(p, "1") == 10 and not p.has_holds() and not p.decrement_holds()
    # change bringing up (metric decrease): held UP calls
    a.adjs[0].metric = 5
    assert not _upd(p, a)[0]
    for _ in range(UP - 1):
        assert p.has_holds() and _metric(p, "1") == 10
        assert not p.decrement_holds()
    assert p.decrement_holds()
    assert not p.has_holds() and _metric(p, "1") == 5
    # an increase is held DOWN calls; zero TTLs apply at once
    a.adjs[0].metric = 7
    assert not _upd(p, a)[0]
    assert _metric(p, "1") == 5
    for _ in range(DOWN):
        p.decrement_holds()
    assert _metric(p, "1") == 7
    a.adjs[0].metric = 9
    assert _upd(p, a, 0, 0)[0] and _metric(p, "1") == 9


def test_new_link_held_down_until_hold_up_expires():
    p = _ls()
    a, b = _pair()
    p.apply(AdjDbStream.from_dbs([a]))
    ch = _upd(p, b, up=3, down=0)  # the link forms with a hold-up TTL
    assert not ch[0] and p.has_holds()
    assert [up for _, _, up in p.links("1")] == [False]
    assert "2" not in _reached(p, "1")
    assert not p.decrement_holds() and not p.decrement_holds()
    assert p.decrement_holds()
    assert [up for _, _, up in p.links("1")] == [True] and not p.has_holds()
    assert "2" in _reached(p, "1")


def _reached(p, root):
    return {ln.split("\t")[0] for ln in p.spf_text(root).splitlines() if ln}


def _ring(n, rng, wmax=9):
    names = [f"n{i:02d}" for i in range(n)]
    adjs = {x: [] for x in names}
    for i in range(n):
        for j in (i + 1, i + 3):
            if j >= n:
                continue
            a, b = names[i], names[j]
            adjs[a].append(create_adjacency(b, f"{a}/{b}", f"{b}/{a}", int(rng.integers(1, wmax + 1))))
            adjs[b].append(create_adjacency(a, f"{b}/{a}", f"{a}/{b}", int(rng.integers(1, wmax + 1))))
    return names, [AdjDb(x, adjs[x], k + 1) for k, x in enumerate(names)]


def _oracle_text(dbs, root):
    o = Oracle()
    o.apply(AdjDbStream.from_dbs(dbs))
    return o.spf_text(root, True)


@pytest.mark.parametrize("seed", range(3))
def test_held_metric_and_overload_changes_spf_vs_oracle(seed):
    """A batch of metric changes (up and down) and a node overload, all held:
    SPF follows the held graph, then each expiry, against the oracle of the
    graph in effect."""
    import copy
    rng = np.random.default_rng(seed)
    names, dbs = _ring(24, rng)
    p = _ls()
    p.apply(AdjDbStream.from_dbs(dbs))
    before = copy.deepcopy(dbs)
    roots = [names[0], names[7], names[13]]
    for r in roots:
        assert p.spf_text(r) == _oracle_text(before, r)
    # node 5 lowers two metrics (held 2 calls), node 11 raises one (held 4),
    # node 17 overloads (held 4)
    d5, d11, d17 = dbs[5], dbs[11], dbs[17]
    for adj in d5.adjs[:2]:
        adj.metric = max(1, adj.metric - 5) if adj.metric > 1 else adj.metric
    d11.adjs[0].metric += 20
    d17.overloaded = True
    for d in (d5, d11, d17):
        _upd(p, d, up=2, down=4)
    for r in roots:
        assert p.spf_text(r) == _oracle_text(before, r), r
    mid = copy.deepcopy(before)
    mid[5] = copy.deepcopy(d5)  # the metric decreases expire after 2 calls
    p.decrement_holds()
    p.decrement_holds()
    for r in roots:
        assert p.spf_text(r) == _oracle_text(mid, r), r
    p.decrement_holds()
    assert p.has_holds()
    p.decrement_holds()  # the raise and the overload expire
    assert not p.has_holds()
    for r in roots:
        assert p.spf_text(r) == _oracle_text(dbs, r), r
