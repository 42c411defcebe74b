"""Weighted derive (ospf_wderive_dev): the rows of leaf roots derived from
their neighbours' distance rows must equal the per-root engine path (and so
the oracle-pinned results) bit for bit -- dist rows, next-hop rows, digests --
on weighted graphs with metrics far above 63, overloaded nodes, down and
parallel links, on the weighted fabric with drains, in hop-count mode, with
byte-wise row ends (V % 4 != 0) and misaligned rows."""
import numpy as np
import pytest
import torch

from graphs import random_stream
from oracle import Oracle
from openr_amd import shard
from openr_amd import topology as T
from openr_amd.adjdb import AdjDbStream
from openr_amd.engine import Engine, EngineError
from openr_amd.linkstate import LinkState

pytestmark = pytest.mark.gpu


def wderive_all(eng, csr, hop=False, offset=0):
    """Cover roots through eng.run (variant chosen by the engine), leaf roots
    derived from their rows. Returns (leaf ids, dist, nh, digests)."""
    dev = torch.device("cuda", 0)
    V = eng.V
    leaf = shard.leaf_set(csr["row_ptr"], csr["col"])
    cover, lr = shard.wderive_plan(np.arange(V, dtype=np.uint32), leaf, csr["row_ptr"],
                                   csr["col"])
    ref = eng.run(cover, max(eng.nh_words(int(r)) for r in cover),
                  hop_count=hop, want_digest=True) if cover.size else None
    pos = np.full(V, 0xFFFFFFFF, np.uint32)
    pos[cover] = np.arange(cover.size, dtype=np.uint32)
    # rows at an offset of `offset` words from a 16-B boundary: byte-wise path
    src = torch.zeros(max(1, cover.size) * V + offset, dtype=torch.int32, device=dev)
    if cover.size:
        src[offset:offset + cover.size * V] = torch.from_numpy(
            ref["dist"].reshape(-1).view(np.int32)).to(dev)
    d_pos = torch.from_numpy(pos.view(np.int32)).to(dev)
    d_r = torch.from_numpy(lr.view(np.int32)).to(dev)
    n = lr.size
    dist = torch.empty(n * V + offset, dtype=torch.int32, device=dev)
    nh = torch.empty(n * V + offset, dtype=torch.int32, device=dev)
    dg = torch.empty((n, 3), dtype=torch.int64, device=dev)
    kmax = int(shard.distinct_neighbors(csr["row_ptr"], csr["col"])[lr].max()) if n else 0
    eng.wderive_dev(d_r.data_ptr(), n, src.data_ptr() + 4 * offset, d_pos.data_ptr(),
                    dist.data_ptr() + 4 * offset, d_nh=nh.data_ptr() + 4 * offset,
                    d_digest=dg.data_ptr(), max_root_neighbors=kmax, hop_count=hop)
    eng.sync()
    return (lr, dist[offset:].cpu().numpy().view(np.uint32).reshape(n, V),
            nh[offset:].cpu().numpy().view(np.uint32).reshape(n, V),
            dg.cpu().numpy().view(np.uint64))


def check_against_engine(stream, hop=False, offset=0, min_leaves=1):
    ls = LinkState()
    ls.apply(stream)
    csr = ls.csr()
    eng = Engine()
    try:
        eng.load(csr)
        lr, dist, nh, dg = wderive_all(eng, csr, hop, offset)
        assert lr.size >= min_leaves
        ref = eng.run(lr, 1, hop_count=hop, want_digest=True)
        assert np.array_equal(dist, ref["dist"])
        assert np.array_equal(nh, ref["nh"].reshape(lr.size, -1))
        assert np.array_equal(dg, ref["digest"])
    finally:
        eng.close()
    return ls, lr, dg


@pytest.mark.parametrize("seed", range(6))
def test_wderive_random_weighted_graphs(seed):
    """Metrics up to 100,000 (far beyond the 63 of the per-root Dial ring),
    overloads, down and parallel links."""
    stream, _ = random_stream(300 + seed, n=80, p=0.06, wmax=100_000)
    check_against_engine(stream, min_leaves=10)


@pytest.mark.parametrize("seed", range(2))
def test_wderive_small_metrics_with_ties(seed):
    """Metrics 1..3: many equal-cost paths, so many tight slots per node."""
    stream, _ = random_stream(400 + seed, n=90, p=0.05, wmax=3, overload=0.2)
    check_against_engine(stream, min_leaves=10)


def test_wderive_hop_count_mode():
    stream, _ = random_stream(500, n=70, p=0.06, wmax=50)
    check_against_engine(stream, hop=True, min_leaves=10)


@pytest.mark.parametrize("offset", [0, 1])
def test_wderive_weighted_fabric_with_drains(offset):
    """Racks derived from their fabric switches' rows (one uniform run per
    pod), with an overloaded fabric switch (a next hop towards itself only),
    an overloaded rack, and a down rack uplink; offset 1 = rows off a 16-B
    boundary (scalar loads / stores)."""
    st = T.fabric(pods=12, planes=8, weighted_seed=11, max_metric=200)
    dbs = st.to_dbs()
    for d in dbs:
        if d.name in ("2-3-1", "3-5-7"):
            d.overloaded = True
        if d.name == "3-4-2":
            d.adjs[0].overloaded = True
    _, lr, dg = check_against_engine(AdjDbStream.from_dbs(dbs), offset=offset, min_leaves=500)


def test_wderive_grid_odd_size_vs_oracle():
    """A weighted grid with V % 4 != 0 (tile ends), compared with the
    reference-shaped oracle as well."""
    st = T.grid(19)
    dbs = st.to_dbs()
    rng = np.random.default_rng(5)
    for d in dbs:
        for a in d.adjs:
            a.metric = int(rng.integers(1, 500))
        if int(d.name) % 11 == 4:
            d.overloaded = True
    st2 = AdjDbStream.from_dbs(dbs)
    ls, lr, dg = check_against_engine(st2, min_leaves=50)
    names = ls.node_names()
    pick = [int(x) for x in lr[:: max(1, lr.size // 6)]]
    want = Oracle(st2).digests([names[i] for i in pick])
    got = dict(zip(lr.tolist(), dg))
    for r, w in zip(pick, want):
        assert np.array_equal(got[r], w), names[r]


def test_wderive_wide_root_is_an_error():
    st = T.fabric(pods=40, planes=1)  # spines with 40 neighbours
    ls = LinkState()
    ls.apply(st)
    eng = Engine()
    try:
        eng.load(ls.csr())
        V = eng.V
        dev = torch.device("cuda", 0)
        src = torch.zeros((V, V), dtype=torch.int32, device=dev)
        pos = torch.from_numpy(np.arange(V, dtype=np.int32)).to(dev)
        r = torch.tensor([ls.node_names().index("1-0-0")], dtype=torch.int32, device=dev)
        dist = torch.empty((1, V), dtype=torch.int32, device=dev)
        eng.wderive_dev(r.data_ptr(), 1, src.data_ptr(), pos.data_ptr(), dist.data_ptr())
        with pytest.raises(EngineError):
            eng.sync()
        with pytest.raises(EngineError):  # a bound above 32 is refused up front
            eng.wderive_dev(r.data_ptr(), 1, src.data_ptr(), pos.data_ptr(), dist.data_ptr(),
                            max_root_neighbors=40)
    finally:
        eng.close()


def test_wderive_missing_neighbour_row_is_an_error():
    st = T.fabric(pods=4, planes=2, weighted_seed=3)
    ls = LinkState()
    ls.apply(st)
    eng = Engine()
    try:
        eng.load(ls.csr())
        V = eng.V
        dev = torch.device("cuda", 0)
        src = torch.zeros((V, V), dtype=torch.int32, device=dev)
        pos = np.arange(V, dtype=np.uint32)
        pos[ls.node_names().index("2-0-1")] = 0xFFFFFFFF  # a fabric switch of rack 3-0-0
        d_pos = torch.from_numpy(pos.view(np.int32)).to(dev)
        r = torch.tensor([ls.node_names().index("3-0-0")], dtype=torch.int32, device=dev)
        dist = torch.empty((1, V), dtype=torch.int32, device=dev)
        eng.wderive_dev(r.data_ptr(), 1, src.data_ptr(), d_pos.data_ptr(), dist.data_ptr())
        with pytest.raises(EngineError):
            eng.sync()
    finally:
        eng.close()


# ---------------------------------------------------------------- cover SPF
def cover_pipeline(eng, csr, check_nh=True):
    """Cover dist rows by the contracted-graph SPF, leaf rows by wderive,
    cover next hops by wderive_wide; returns {root: (dist, nh, digest)}."""
    dev = torch.device("cuda", 0)
    V = eng.V
    rp, col = csr["row_ptr"], csr["col"]
    leaf = shard.leaf_set(rp, col)
    eng.cover_prepare(leaf)
    cover = np.nonzero(~leaf)[0].astype(np.uint32)
    lr = np.nonzero(leaf)[0].astype(np.uint32)
    pos = np.empty(V, np.uint32)
    pos[cover] = np.arange(cover.size, dtype=np.uint32)
    pos[lr] = cover.size + np.arange(lr.size, dtype=np.uint32)
    slab = torch.empty((V, V), dtype=torch.int32, device=dev)
    d_pos = torch.from_numpy(pos.view(np.int32)).to(dev)
    d_c = torch.from_numpy(cover.view(np.int32)).to(dev)
    d_l = torch.from_numpy(lr.view(np.int32)).to(dev)
    eng.cover_dist_dev(d_c.data_ptr(), cover.size, slab.data_ptr())
    nbrs = shard.distinct_neighbors(rp, col)
    out = {}
    if lr.size:
        lnh = torch.empty((lr.size, V), dtype=torch.int32, device=dev)
        ldg = torch.empty((lr.size, 3), dtype=torch.int64, device=dev)
        eng.wderive_dev(d_l.data_ptr(), lr.size, slab.data_ptr(), d_pos.data_ptr(),
                        slab[cover.size].data_ptr(), d_nh=lnh.data_ptr(), d_digest=ldg.data_ptr(),
                        max_root_neighbors=int(nbrs[lr].max()))
        eng.sync()
        ln, lg = lnh.cpu().numpy().view(np.uint32), ldg.cpu().numpy().view(np.uint64)
        for j, r in enumerate(lr):
            out[int(r)] = (None, ln[j].reshape(V, 1), lg[j])
    if check_nh:
        for W in sorted(set(np.maximum(1, (nbrs[cover] + 31) // 32).tolist())):
            grp = cover[(np.maximum(1, (nbrs[cover] + 31) // 32) == W)]
            if not grp.size:
                continue
            d_g = torch.from_numpy(grp.view(np.int32)).to(dev)
            nh = torch.empty((grp.size, V, W), dtype=torch.int32, device=dev)
            dg = torch.empty((grp.size, 3), dtype=torch.int64, device=dev)
            eng.wderive_wide_dev(d_g.data_ptr(), grp.size, W, slab.data_ptr(), d_pos.data_ptr(),
                                 nh.data_ptr(), d_digest=dg.data_ptr())
            eng.sync()
            n_h, g_h = nh.cpu().numpy().view(np.uint32), dg.cpu().numpy().view(np.uint64)
            for j, r in enumerate(grp):
                out[int(r)] = (None, n_h[j], g_h[j])
    eng.sync()
    dist = slab.cpu().numpy().view(np.uint32)
    return {r: (dist[pos[r]], nh, dg) for r, (_, nh, dg) in out.items()}, cover, dist, pos


def check_cover(stream, sample=0):
    """Every cover row against the engine; every root's (or `sample` random
    roots' plus every root with > 4 next-hop words) dist / next hops / digest
    against the per-root engine path."""
    ls = LinkState()
    ls.apply(stream)
    csr = ls.csr()
    eng = Engine()
    try:
        eng.load(csr)
        got, cover, dist, pos = cover_pipeline(eng, csr)
        ref = eng.run(cover, max(eng.nh_words(int(r)) for r in cover), want_nh=False)
        assert np.array_equal(dist[pos[cover]], ref["dist"])  # every cover row
        keys = sorted(got)
        if sample:
            rng = np.random.default_rng(3)
            keys = sorted(set(rng.choice(keys, min(sample, len(keys)), replace=False).tolist()) |
                          {r for r in keys if got[r][1].shape[1] > 4})
        for r in keys:
            d, nh, dg = got[r]
            W = nh.shape[1]
            want = eng.run([r], W, want_digest=True)
            assert np.array_equal(d, want["dist"][0]), r
            assert np.array_equal(nh, want["nh"][0]), r
            assert np.array_equal(dg, want["digest"][0]), r
    finally:
        eng.close()
    return ls, got


@pytest.mark.parametrize("seed", range(5))
def test_cover_spf_random_weighted_graphs(seed):
    """Contracted-graph SPF of the cover + derived leaves + cover next hops,
    on graphs with overloads, down and parallel links, metrics up to 60,000."""
    stream, _ = random_stream(600 + seed, n=90, p=0.05, wmax=60_000)
    check_cover(stream)


def test_cover_spf_ties():
    stream, _ = random_stream(700, n=100, p=0.05, wmax=3, overload=0.2)
    check_cover(stream)


def test_cover_spf_weighted_fabric_with_drains_vs_oracle():
    st = T.fabric(pods=12, planes=8, weighted_seed=11, max_metric=200)
    dbs = st.to_dbs()
    for d in dbs:
        if d.name in ("2-3-1", "3-5-7", "3-6-1"):
            d.overloaded = True
        if d.name in ("3-4-2", "2-7-7"):
            d.adjs[0].overloaded = True
    st2 = AdjDbStream.from_dbs(dbs)
    ls, got = check_cover(st2)
    names = ls.node_names()
    pick = ["2-3-1", "2-0-0", "3-5-7", "3-4-2", "2-7-7", "3-11-47"]
    want = Oracle(st2).digests(pick)
    for nm, w in zip(pick, want):
        assert np.array_equal(got[names.index(nm)][2], w), nm


def test_cover_graph_goes_stale_on_updates():
    stream, _ = random_stream(710, n=40, p=0.1, wmax=50)
    ls = LinkState()
    ls.apply(stream)
    csr = ls.csr()
    eng = Engine()
    try:
        eng.load(csr)
        leaf = shard.leaf_set(csr["row_ptr"], csr["col"])
        eng.cover_prepare(leaf)
        V = eng.V
        dev = torch.device("cuda", 0)
        r = int(np.nonzero(~leaf)[0][0])
        d_r = torch.tensor([r], dtype=torch.int32, device=dev)
        dist = torch.empty((1, V), dtype=torch.int32, device=dev)
        eng.cover_dist_dev(d_r.data_ptr(), 1, dist.data_ptr())
        eng.sync()
        eng.update_nodes([r], [1], version=7)
        with pytest.raises(EngineError):
            eng.cover_dist_dev(d_r.data_ptr(), 1, dist.data_ptr())
        bad = leaf.copy()
        bad[:] = True  # adjacent leaves
        with pytest.raises(EngineError):
            eng.cover_prepare(bad)
    finally:
        eng.close()


@pytest.mark.parametrize("pods,planes", [(150, 2), (300, 1)])
def test_cover_spf_wide_spines(pods, planes):
    """Spines with 150 / 300 neighbours (5 / 10 next-hop words): the lane-per-
    word kernel, runs of one plane's spines, a drained fabric switch, an
    overloaded spine adjacency and a down link."""
    st = T.fabric(pods=pods, planes=planes, weighted_seed=5, max_metric=300)
    dbs = st.to_dbs()
    for d in dbs:
        if d.name in ("2-3-0", "2-140-0"):
            d.overloaded = True
        if d.name in ("1-0-5", "1-0-30"):
            d.adjs[7].overloaded = True
    check_cover(AdjDbStream.from_dbs(dbs), sample=200)
