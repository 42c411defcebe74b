"""Full-size parity of the all-sources sweeps under the reference's edge cases
(VERDICT r03 next #2): the F100k fabric with drained (overloaded) nodes and
down links on the unit-metric derive sweep, and the weighted F100k (metrics
1..64, seed 7) with and without drains on the weighted cover sweep.

Each sweep's per-root digests are checked against the CSR-Dijkstra CPU
restatement (oracle/, test infrastructure) on every spine, every drained node,
a sample of the nodes incident to a down link and 256 random fabric / rack
switches; whole dist + next-hop rows of >= 32 roots per width class are
compared with the per-batch engine path; every root's reached count is checked
against a host BFS of the usable graph.

Reference semantics: LinkState::runSpf (openr/decision/LinkState.cpp:836-911),
overloaded nodes recorded but never relaying (:859-866), Link::isUp
(:242-245)."""
import time

import numpy as np
import pytest

from graphs import drained_fabric
from oracle import Oracle
from openr_amd import topology as T
from openr_amd.engine import Engine, Sweep
from openr_amd.linkstate import LinkState

pytestmark = pytest.mark.gpu

T0 = time.time()


def note(msg):
    print(f"[{time.time() - T0:7.1f}s] {msg}", flush=True)


def reached_counts(csr, roots):
    """Nodes each root reaches over usable links, non-transit nodes relaying
    only as the root (scipy BFS over the transit subgraph + one hop)."""
    from scipy.sparse import csr_matrix
    from scipy.sparse.csgraph import connected_components
    V = csr["row_ptr"].size - 1
    rp = csr["row_ptr"].astype(np.int64)
    src = np.repeat(np.arange(V), np.diff(rp))
    col = csr["col"].astype(np.int64)
    up = csr["edge_up"].astype(bool)
    nt = csr["no_transit"].astype(bool)
    keep = up & ~nt[src] & ~nt[col]
    g = csr_matrix((np.ones(int(keep.sum()), np.int8), (src[keep], col[keep])), shape=(V, V))
    _, comp = connected_components(g, directed=False)
    # per component of the transit subgraph: its transit nodes and the
    # non-transit nodes one usable link away (reached, never relaying)
    size = np.bincount(comp[~nt], minlength=comp.max() + 1)
    e = up & ~nt[src] & nt[col]
    ntadj = {}
    for k, x in set(zip(comp[src[e]].tolist(), col[e].tolist())):
        ntadj.setdefault(k, set()).add(x)
    out = []
    for r in roots:
        r = int(r)
        if not nt[r]:
            out.append(int(size[comp[r]]) + len(ntadj.get(comp[r], ())))
            continue
        # an overloaded root relays its own links: the components of its
        # transit neighbours, their non-transit neighbours, its own neighbours
        lo, hi = rp[r], rp[r + 1]
        nb = {int(x) for x, u in zip(col[lo:hi], up[lo:hi]) if u}
        ks = {int(comp[x]) for x in nb if not nt[x]}
        seen = {r} | {x for x in nb if nt[x]}
        for k in ks:
            seen |= ntadj.get(k, set())
        out.append(sum(int(size[k]) for k in ks) + len(seen))
    return np.array(out)


def check_sweep(stream, want_mode, hop=False, seed=0x5EED, extra=()):
    o, p = Oracle(), LinkState()
    assert o.apply(stream) == p.apply(stream)
    note("ingested")
    names = p.node_names()
    V = len(names)
    csr = p.csr()
    eng = Engine()
    eng.load(csr)
    sw = Sweep(eng, hop_count=hop)
    assert sw.mode == want_mode
    assert sorted(sw.roots.tolist()) == list(range(V))
    sw.run()
    eng.sync()
    d = np.zeros((V, 3), np.uint64)
    sw._check(sw._L.ospf_sweep_digests_host(sw._h, d.ctypes.data))
    got = np.zeros_like(d)
    got[sw.roots] = d
    note(f"sweep ({sw.mode}) digests")
    role = np.array([int(n.split("-")[0]) for n in names])
    rng = np.random.default_rng(seed)
    nt = np.nonzero(csr["no_transit"])[0]
    rp = csr["row_ptr"].astype(np.int64)
    src = np.repeat(np.arange(V), np.diff(rp))
    down_nodes = np.unique(src[csr["edge_up"] == 0])
    inc = np.sort(rng.choice(down_nodes, min(512, down_nodes.size), replace=False)) \
        if down_nodes.size else np.zeros(0, np.int64)
    spines = np.nonzero(role == 1)[0]
    fsw = np.sort(rng.choice(np.nonzero(role == 2)[0], 256, replace=False))
    rsw = np.sort(rng.choice(np.nonzero(role == 3)[0], 256, replace=False))
    strat = np.unique(np.concatenate([spines, nt, inc, fsw, rsw, np.asarray(extra, np.int64)]))
    want = o.fast_digests([names[i] for i in strat], not hop, threads=16)
    note(f"CSR-Dijkstra digests of {strat.size} roots ({nt.size} drained, {inc.size} "
         f"incident to a down link)")
    bad = [names[r] for j, r in enumerate(strat) if not np.array_equal(got[r], want[j])]
    assert not bad, (len(bad), bad[:8])
    # reached count of every root (size-independent property over all V runs)
    chk = np.unique(np.concatenate([strat, rng.choice(V, 2048, replace=False)]))
    assert np.array_equal(got[chk, 0].astype(np.int64), reached_counts(csr, chk))
    note("reached counts")
    # whole rows of >= 32 roots per width class == the per-batch engine path
    words = np.array([eng.nh_words(int(r)) for r in range(V)])
    for W in sorted(set(words.tolist())):
        grp = np.nonzero(words == W)[0]
        few = np.sort(rng.choice(grp, min(32, grp.size), replace=False)).astype(np.uint32)
        # the class's drained roots and roots next to a down link first
        spec = np.intersect1d(grp, np.concatenate([nt, inc]))[:16].astype(np.uint32)
        few = np.unique(np.concatenate([spec, few]))[:48]
        ref = eng.run(few, W, hop_count=hop, want_digest=True)
        dist, nh = sw.rows(few, W)
        assert np.array_equal(dist, ref["dist"]), W
        assert np.array_equal(nh, ref["nh"]), W
        assert np.array_equal(got[few], ref["digest"]), W
    note("rows == batch path")
    sw.close()
    eng.close()


@pytest.mark.timeout(900)
def test_f100k_drained_unit_derive_sweep():
    """Unit-metric F100k with 2 % drained nodes and 1 % of the adjacencies
    reported overloaded: twin classes split (racks with a down link leave
    their pod's class), leaf groups turn non-uniform, non-transit slots."""
    check_sweep(drained_fabric(1781, 8, seed=11, drain=0.02, down=0.01), "derive")


@pytest.mark.timeout(900)
def test_f100k_weighted_cover_sweep():
    """The weighted F100k (metrics 1..64, seed 7): cover SPF + closure, leaf
    rows, fabric-switch and spine next hops (bench.py --topology
    fabric100k-w)."""
    check_sweep(T.fabric(pods=1781, planes=8, weighted_seed=7), "wcover")


@pytest.mark.timeout(900)
def test_f100k_weighted_drained_cover_sweep():
    """The weighted F100k with 2 % drained nodes and 1 % down adjacencies."""
    check_sweep(drained_fabric(1781, 8, seed=12, drain=0.02, down=0.01, weighted_seed=7),
                "wcover")


def triangle_and_tight(csr, root, dist, nh_bits_ok=None):
    """Size-independent checks of one full dist row: every usable edge u -> v
    out of a relaying node satisfies dist(v) <= dist(u) + w (triangle), and
    every reached v != root has a tight in-edge from a relaying node (the
    shortest path's last hop). Relaying: transit, or the root itself."""
    V = csr["row_ptr"].size - 1
    rp = csr["row_ptr"].astype(np.int64)
    src = np.repeat(np.arange(V), np.diff(rp))
    col = csr["col"].astype(np.int64)
    w = csr["metric"].astype(np.int64)
    up = csr["edge_up"].astype(bool)
    relay = ~csr["no_transit"].astype(bool)
    relay[root] = True
    d = dist.astype(np.int64)
    inf = np.int64(0xFFFFFFFF)
    ok = up & relay[src] & (d[src] != inf)
    assert np.all(d[col[ok]] <= d[src[ok]] + w[ok]), "triangle"
    tight = ok & (d[col] == d[src] + w)
    has = np.zeros(V, bool)
    has[col[tight]] = True
    reached = d != inf
    reached[root] = False
    assert np.all(has[reached]), "tight last hop"
    assert d[root] == 0


@pytest.mark.timeout(900)
def test_m1m_wmulti_sweep_part():
    """M1M (1M-node random-geometric mesh, metrics 1..16): the middle part of
    a 122-part all-sources partition on the multi-root traversal (WMULTI:
    groups of 32 roots, [node][root] state) + derived leaf rows and next
    hops: 64 roots' digests == the CSR-Dijkstra restatement, whole rows of 32
    roots == the per-root batch path, triangle + tight-last-hop checks on 4
    full rows."""
    st = T.mesh(1_000_000, seed=42)
    p = LinkState()
    p.apply(st)
    names = p.node_names()
    csr = p.csr()
    note("ingested")
    eng = Engine()
    eng.load(csr)
    sw = Sweep(eng, part=61, n_parts=122, mode="wmulti", hip_graph=False)
    n = sw.n_roots
    assert 7000 < n < 9500, n
    sw.run()
    eng.sync()
    d = np.zeros((n, 3), np.uint64)
    sw._check(sw._L.ospf_sweep_digests_host(sw._h, d.ctypes.data))
    got = dict(zip(sw.roots.tolist(), d))
    note(f"wmulti part: {n} roots, {sw.n_rows} rows")
    roots = np.sort(sw.roots)
    rng = np.random.default_rng(4)
    pick = np.sort(rng.choice(roots, 64, replace=False))
    o = Oracle(st)
    want = o.fast_digests([names[i] for i in pick], True, threads=16)
    bad = [names[r] for j, r in enumerate(pick) if not np.array_equal(got[int(r)], want[j])]
    assert not bad, (len(bad), bad[:8])
    note("64 roots == CSR-Dijkstra")
    few = np.sort(rng.choice(roots, 32, replace=False)).astype(np.uint32)
    words = np.array([eng.nh_words(int(r)) for r in few])
    for W in sorted(set(words.tolist())):
        grp = few[words == W]
        ref = eng.run(grp, W, want_digest=True)
        dist, nh = sw.rows(grp, W)
        assert np.array_equal(dist, ref["dist"]), W
        assert np.array_equal(nh, ref["nh"]), W
        for j, r in enumerate(grp.tolist()):
            assert np.array_equal(got[r], ref["digest"][j])
    note("32 roots' rows == batch path")
    for r in few[:4].tolist():
        dist, _ = sw.rows(np.array([r], np.uint32), max(1, eng.nh_words(r)))
        triangle_and_tight(csr, r, dist[0])
    note("triangle + tight last hops")
    sw.close()
    eng.close()



def text_fields_of_row(names, nbrs, dist, nh):
    """{name: (metric, sorted next-hop names)} of one root's engine rows: the
    first two fields of the getSpfResult text (DESIGN.md §Result text)."""
    out = {}
    inf = np.uint32(0xFFFFFFFF)
    for v in np.nonzero(dist != inf)[0].tolist():
        hops = []
        for w in range(nh.shape[1]):
            x = int(nh[v, w])
            while x:
                b = (x & -x).bit_length() - 1
                hops.append(names[int(nbrs[32 * w + b])])
                x &= x - 1
        out[names[v]] = (int(dist[v]), tuple(sorted(hops)))
    return out


@pytest.mark.timeout(1200)
def test_m1m_wderive_sweep_part():
    """The M1M path bench.py --topology mesh1m measures:
    the middle part of the 122-part all-sources partition on the weighted
    derive sweep (sweep:wderive -- per-root Dial for the part's cover roots,
    leaf rows derived from their neighbours' rows). 64 roots' digests == the
    CSR-Dijkstra restatement; every node's metric and next-hop set of 2 roots
    (a leaf and a cover root) == the reference-shaped runSpf text
    (LinkState.cpp:836-911); triangle + tight-last-hop checks on 4 rows."""
    from oracle import parse_spf_text
    st = T.mesh(1_000_000, seed=42)
    o, p = Oracle(), LinkState()
    assert o.apply(st) == p.apply(st)
    names = p.node_names()
    csr = p.csr()
    note("ingested")
    eng = Engine()
    eng.load(csr)
    sw = Sweep(eng, part=61, n_parts=122, mode="wderive", hip_graph=False)
    assert sw.mode == "wderive"
    n = sw.n_roots
    assert 7000 < n < 9500, n
    sw.run()
    eng.sync()
    d = np.zeros((n, 3), np.uint64)
    sw._check(sw._L.ospf_sweep_digests_host(sw._h, d.ctypes.data))
    got = dict(zip(sw.roots.tolist(), d))
    note(f"wderive part: {n} roots, {sw.n_rows} rows")
    roots = np.sort(sw.roots)
    rng = np.random.default_rng(5)
    pick = np.sort(rng.choice(roots, 64, replace=False))
    want = o.fast_digests([names[i] for i in pick], True, threads=16)
    bad = [names[r] for j, r in enumerate(pick) if not np.array_equal(got[int(r)], want[j])]
    assert not bad, (len(bad), bad[:8])
    note("64 roots == CSR-Dijkstra")
    # a leaf root (<= 32 neighbours, derived) and the widest root of the part
    deg = np.array([eng.root_neighbors(int(r)).size for r in roots])
    two = [int(roots[int(np.argmin(deg))]), int(roots[int(np.argmax(deg))])]
    for r in two:
        W = max(1, eng.nh_words(r))
        dist, nh = sw.rows(np.array([r], np.uint32), W)
        mine = text_fields_of_row(names, eng.root_neighbors(r), dist[0], nh[0])
        ref = {k: (v[0], tuple(sorted(v[1]))) for k, v in
               parse_spf_text(o.spf_text(names[r])).items()}
        assert mine == ref, names[r]
        note(f"{names[r]}: {len(mine)} nodes' metric + next hops == reference-shaped runSpf")
    for r in pick[:4].tolist():
        dist, _ = sw.rows(np.array([r], np.uint32), max(1, eng.nh_words(r)))
        triangle_and_tight(csr, r, dist[0])
    note("triangle + tight last hops")
    sw.close()
    eng.close()


@pytest.mark.timeout(900)
def test_f100k_weighted_sweep_whole_rows_vs_scipy():
    """Whole dist + next-hop rows of the weighted F100k (metrics 1..64)
    all-sources sweep (cover SPF + derived leaves) against an independent
    solver: scipy's Dijkstra from the root and from each of its neighbours,
    next hops = the neighbours n with w(r, n) + dist(n, v) == dist(r, v)
    (LinkState.cpp:885-901; every node is transit here). Racks, fabric
    switches and a spine (56 next-hop words); the reference-shaped runSpf
    text takes minutes per root at this size with metrics."""
    from scipy.sparse import csr_matrix
    from scipy.sparse.csgraph import dijkstra
    st = T.fabric(pods=1781, planes=8, weighted_seed=7)
    ls = LinkState()
    ls.apply(st)
    csr = ls.csr()
    names = ls.node_names()
    V = len(names)
    eng = Engine()
    eng.load(csr)
    sw = Sweep(eng)
    sw.run()
    eng.sync()
    note(f"weighted F100k sweep ({sw.mode})")
    rp, col = csr["row_ptr"].astype(np.int64), csr["col"].astype(np.int64)
    up = csr["edge_up"] != 0
    row = np.repeat(np.arange(V), np.diff(rp))
    # parallel links: the smallest metric per (row, neighbour)
    key = row[up] * V + col[up]
    order = np.lexsort((csr["metric"][up], key))
    first = np.ones(order.size, bool)
    first[1:] = key[order][1:] != key[order][:-1]
    sel = order[first]
    G = csr_matrix((csr["metric"][up][sel].astype(np.float64), (row[up][sel], col[up][sel])), shape=(V, V))
    for r in [names.index(x) for x in ("3-2-2", "3-1200-40", "2-17-3", "2-1500-0", "1-5-30")]:
        nb = np.unique(col[rp[r]:rp[r + 1]])
        nb = nb[nb != r]
        W = eng.nh_words(int(r))
        dist, nh = sw.rows(np.array([r], np.uint32), W)
        D = dijkstra(G, indices=np.concatenate([[r], nb]))
        d0 = np.where(np.isinf(D[0]), 0xFFFFFFFF, D[0]).astype(np.uint64)
        assert np.array_equal(dist[0].astype(np.uint64), d0), names[r]
        want = np.zeros((V, W), np.uint32)
        for k, n in enumerate(nb):
            wr = G[r, n]
            if wr == 0:
                continue  # no up link to n
            tight = np.isfinite(D[0]) & (wr + D[1 + k] == D[0])
            tight[r] = False
            want[tight, k >> 5] |= np.uint32(1 << (k & 31))
        assert np.array_equal(nh[0], want), names[r]
        note(f"weighted F100k whole rows of {names[r]} == scipy Dijkstra")
    sw.close()
    eng.close()
