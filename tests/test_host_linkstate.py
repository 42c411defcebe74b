"""CPU: host-side LinkState mirror (ingest, link identity/order, change
flags, CSR snapshot) against the reference fixtures and the oracle.
No SPF here: SPF needs the MI355X engine (tests/test_gpu_parity.py)."""
import numpy as np
import pytest

from golden_eval import ProductLS, load_fixtures, run_fixture
from oracle import Oracle
from openr_amd import topology as T
from openr_amd.adjdb import AdjDb, AdjDbStream, create_adjacency
from openr_amd.linkstate import LinkState, LinkStateError

FIXTURES = load_fixtures()


@pytest.mark.parametrize("fx", FIXTURES, ids=[f["name"] for f in FIXTURES])
def test_ingest_matches_reference_fixture(fx):
    run_fixture(fx, ProductLS, spf=False)


def _random_stream(seed, n=40, p=0.15, parallel=0.2, overload=0.1, down=0.1, wmax=20):
    rng = np.random.default_rng(seed)
    names = [f"r{int(x)}" for x in rng.permutation(10 * n)[:n]]
    adjs = {nm: [] for nm in names}
    k = 0
    for i in range(n):
        for j in range(i + 1, n):
            if rng.random() > p:
                continue
            reps = 2 if rng.random() < parallel else 1
            for r in range(reps):
                a, b = names[i], names[j]
                ia, ib = f"{a}-{b}-{k}", f"{b}-{a}-{k}"
                k += 1
                dn = rng.random() < down
                adjs[a].append(create_adjacency(b, ia, ib, int(rng.integers(1, wmax + 1)),
                                                overloaded=dn))
                adjs[b].append(create_adjacency(a, ib, ia, int(rng.integers(1, wmax + 1))))
    dbs = [AdjDb(nm, adjs[nm], i + 1, overloaded=bool(rng.random() < overload))
           for i, nm in enumerate(names)]
    order = rng.permutation(n)
    return AdjDbStream.from_dbs([dbs[i] for i in order]), names


def _links(ls, node):
    return [(k, m, up) for k, m, up in ls.links(node)]


@pytest.mark.parametrize("seed", range(6))
def test_ingest_random_graph_matches_oracle(seed):
    st, names = _random_stream(seed)
    o, p = Oracle(), LinkState()
    assert o.apply(st) == p.apply(st)
    assert o.num_links() == p.num_links() and o.num_nodes() == p.num_nodes()
    for nm in names:
        ol = [tuple(ln.split("\t")) for ln in o.links_text(nm).splitlines()]
        pl = [(k, str(m), "1" if up else "0") for k, m, up in _links(p, nm)]
        # same links, same iteration order (folly-hash unordered_set order)
        assert ol == pl, nm
        assert o.is_overloaded(nm) == p.is_overloaded(nm)


def test_csr_snapshot_invariants():
    st, names = _random_stream(11, n=60)
    p = LinkState(stream=st)
    c = p.csr()
    V = len(c["row_ptr"]) - 1
    assert V == p.num_nodes()
    ids = p.node_names()
    assert ids == sorted(ids)  # node id = rank of the name (byte order)
    rp, col, tw = c["row_ptr"], c["col"], c["twin"]
    for u in range(V):
        row = col[rp[u]:rp[u + 1]]
        assert np.all(np.diff(row.astype(np.int64)) >= 0)
        for e in range(rp[u], rp[u + 1]):
            t = tw[e]
            assert tw[t] == e and col[t] == u and c["link_id"][t] == c["link_id"][e]
            assert c["edge_up"][t] == c["edge_up"][e]
    # link_rank = position in linksFromNode iteration; metric from the row node
    for u in range(V):
        order = _links(p, ids[u])
        for e in range(rp[u], rp[u + 1]):
            key, m, up = order[c["link_rank"][e]]
            assert m == c["metric"][e] and up == bool(c["edge_up"][e])
        assert sorted(c["link_rank"][rp[u]:rp[u + 1]].tolist()) == list(range(rp[u + 1] - rp[u]))
    assert c["no_transit"].tolist() == [int(p.is_overloaded(n)) for n in ids]


def test_grid_snapshot_shape():
    p = LinkState(stream=T.grid(10))
    c = p.csr()
    assert len(c["row_ptr"]) - 1 == 100 and len(c["col"]) == 360


def test_fabric_generator_shape():
    st = T.fabric(pods=4, planes=8)
    p = LinkState(stream=st)
    # 8*36 ssw + 4*8 fsw + 4*48 rsw; links: fsw-ssw 4*8*36 + rsw-fsw 4*48*8
    assert p.num_nodes() == 288 + 32 + 192
    assert p.num_links() == 4 * 8 * 36 + 4 * 48 * 8
    q = LinkState(stream=T.fabric(pods=4, planes=8, reference_quirk=True))
    # quirk: spines connect to pod 0 only (RoutingBenchmarkUtils.cpp:324-335)
    assert q.num_links() == 8 * 36 + 4 * 48 * 8


def test_spf_without_device_fails_loudly():
    import ctypes
    from openr_amd import _native as N
    h = ctypes.c_void_p()
    rc = N.engine().ospf_open(0, ctypes.byref(h))
    if rc == 0:  # a GPU is present: nothing to check here
        N.engine().ospf_close(h)
        pytest.skip("HIP device present")
    assert rc == N.OSPF_E_DEVICE
    p = LinkState(stream=T.grid(3))
    with pytest.raises(LinkStateError, match="engine"):
        p.spf("0")


def _links_state(p, names):
    return {n: p._take(p._L.odl_links_text(p._h, n.encode())) for n in names}


@pytest.mark.parametrize("seed", range(3))
def test_bulk_ingest_equals_one_by_one(seed, monkeypatch):
    """A batch of >= 64 new nodes takes LinkState::updateAdjacencyDatabases'
    threaded path: the same change records, the same link sets in the same
    linksFromNode iteration order (which fixes pathLinks / KSP2 order), the
    same CSR as applying the databases one by one; also when part of the
    graph is known before the batch, and for a batch that repeats a node
    (sequential fallback)."""
    from graphs import random_stream
    st, names = random_stream(seed, n=160, p=0.05)
    dbs = st.to_dbs()
    monkeypatch.setenv("ODL_NO_BULK_INGEST", "1")
    ref = LinkState()
    ch_ref = ref.apply(st)
    monkeypatch.delenv("ODL_NO_BULK_INGEST")
    got = LinkState()
    ch = got.apply(st)
    assert ch == ch_ref
    assert _links_state(got, names) == _links_state(ref, names)
    a, b = got.csr(), ref.csr()
    assert all(np.array_equal(a[k], b[k]) for k in a)
    # 40 nodes known first (one by one), then a bulk batch of the other 120
    part = LinkState()
    part.apply(AdjDbStream.from_dbs(dbs[:40]))
    ch2 = part.apply(AdjDbStream.from_dbs(dbs[40:]))
    assert ch2 == ch_ref[40:]
    assert _links_state(part, names) == _links_state(ref, names)
    # a batch that updates known nodes again: one by one, same state
    again = part.apply(AdjDbStream.from_dbs(dbs[:100]))
    assert all(not c[0] for c in again)  # nothing changed
    assert _links_state(part, names) == _links_state(ref, names)


def test_bulk_ingest_matches_oracle():
    """The threaded batch path against the reference-shaped restatement
    (oracle/: the reference's own one-by-one ingest): change records, link
    counts and every node's linksFromNode order on a 640-node fabric with
    drains and down links and on a 200-node random graph."""
    from graphs import drained_fabric, random_stream
    for st in (drained_fabric(12, 4, seed=2), random_stream(9, n=200, p=0.04)[0]):
        o, p = Oracle(), LinkState()
        assert o.apply(st) == p.apply(st)
        assert o.num_links() == p.num_links() and o.num_nodes() == p.num_nodes()
        for nm in p.node_names():
            ol = [tuple(ln.split("\t")) for ln in o.links_text(nm).splitlines()]
            pl = [(k, str(m), "1" if up else "0") for k, m, up in _links(p, nm)]
            assert ol == pl, nm


def _host_product():
    p = LinkState()
    p.set_host_spf(True)  # the product's C++ LinkState + SpfSolver, SPF on the host path
    return p


ROUTE_FIXTURES = [f for f in FIXTURES if "route" in f["name"] or "mpls" in f["name"]]


@pytest.mark.parametrize("fx", ROUTE_FIXTURES, ids=[f["name"] for f in ROUTE_FIXTURES])
def test_route_fixtures_through_product_host_spf(fx):
    """The reference's route fixtures (incl. Decision.BestRouteSelection and
    the mixed-type case, DecisionTest.cpp:1240-1384,7203-7290) through the
    C++ odl::SpfSolver on the host SPF path; -m gpu runs the same on the
    engine (test_gpu_parity.py::test_reference_fixture_on_gpu)."""
    assert run_fixture(fx, _host_product) > 0
