"""Synthetic link-state topologies, emitted as AdjacencyDatabase update streams.

* :func:`grid`   — RoutingBenchmarkUtils.cpp:134-184,211-299 (``createGrid``):
  names ``"{r*n+c}"``, adjacency order right, left, up, down, ifName
  ``if_{me}_{other}``, metric 1, nodeLabel id+1, adjLabel 100001+other.
* :func:`fabric` — RoutingBenchmarkUtils.cpp:306-481 (``createFabric``): SSW
  ``"1-{plane}-{i}"``, FSW ``"2-{pod}-{plane}"``, RSW ``"3-{pod}-{i}"``,
  ``if_{me}_{other}``. ``reference_quirk=True`` reproduces the reference's SSW
  ``emplace`` quirk (RoutingBenchmarkUtils.cpp:324-335: only pod 0 wins, so
  spines connect to pod 0 only); the default is the intended topology.
* :func:`mesh`   — Terragraph-style random geometric mesh:
  uniform points (seed), radius sqrt(8/(pi V)), largest component, names
  ``m%07d``, metric max(1, floor(rtt_us/100)) with rtt_us = 100 + 1500 d/r
  (LinkMonitor.cpp:32-34 metric rule).

Large topologies are built column-wise with numpy (no per-adjacency Python
objects) so F100k (2.4M adjacencies) generates in a few seconds.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from .adjdb import AdjDb, AdjDbStream, create_adjacency

SSW, FSW, RSW = 1, 2, 3
SSW_PER_PLANE = 36  # RoutingBenchmarkUtils.h:94
RSW_PER_POD = 48    # RoutingBenchmarkUtils.h:95


def _stream_from_edges(names: Sequence[str], labels: np.ndarray, src: np.ndarray,
                       dst: np.ndarray, metric: np.ndarray, adj_label: np.ndarray,
                       order: Optional[np.ndarray] = None) -> AdjDbStream:
    """Build a stream where node i advertises one adjacency per directed edge
    (src==i), in the given per-node order (edges already grouped by src in
    advertisement order), ifName ``if_{me}_{other}``.

    ``order``: permutation of node indices giving the database ingest order.
    """
    V = len(names)
    E = src.size
    # strings: node names [0, V), then one ifName per directed edge [V, V+E)
    nl = list(names)
    strings = nl + [f"if_{nl[a]}_{nl[b]}" for a, b in zip(src.tolist(), dst.tolist())]
    # reverse edge index: for edge (a->b) find (b->a); pair by sorted keys
    key_f = src.astype(np.int64) * V + dst
    key_r = dst.astype(np.int64) * V + src
    of = np.argsort(key_f, kind="stable")
    pos = np.searchsorted(key_f[of], key_r)
    if np.any(pos >= E) or np.any(key_f[of][np.minimum(pos, E - 1)] != key_r):
        raise ValueError("every edge needs a reverse edge")
    rev = of[pos]
    # group edges by src (stable keeps advertisement order)
    by_src = np.argsort(src, kind="stable")
    counts = np.bincount(src, minlength=V)
    starts = np.zeros(V + 1, np.int64)
    np.cumsum(counts, out=starts[1:])
    if order is None:
        order = np.arange(V)
    # adjacency columns in ingest order
    rank = np.empty(V, np.int64)
    rank[order] = np.arange(V)
    sel = by_src[np.argsort(rank[src[by_src]], kind="stable")] if E else np.zeros(0, np.int64)
    db_off = np.zeros(V + 1, np.uint64)
    np.cumsum(counts[order], out=db_off[1:])
    cols = dict(
        db_name=order.astype(np.uint32),
        db_overloaded=np.zeros(V, np.uint8),
        db_node_label=labels[order].astype(np.int32),
        db_delete=np.zeros(V, np.uint8),
        db_adj_off=db_off,
        adj_other=dst[sel].astype(np.uint32),
        adj_if=(V + sel).astype(np.uint32),
        adj_other_if=(V + rev[sel]).astype(np.uint32),
        adj_metric=metric[sel].astype(np.int32),
        adj_label=adj_label[sel].astype(np.int32),
        adj_overloaded=np.zeros(sel.size, np.uint8),
        adj_weight=np.ones(sel.size, np.int64),
        adj_only_used_by_other=np.zeros(sel.size, np.uint8),
    )
    return AdjDbStream(strings, cols)


def grid(n: int, weighted_seed: Optional[int] = None, max_metric: int = 64) -> AdjDbStream:
    """n x n grid (createGrid). Optional random directed metrics in [1, max_metric]."""
    ids = np.arange(n * n)
    r, c = ids // n, ids % n
    src, dst = [], []
    for dr, dc in ((0, 1), (0, -1), (-1, 0), (1, 0)):  # right, left, up, down
        rr, cc = r + dr, c + dc
        ok = (rr >= 0) & (rr < n) & (cc >= 0) & (cc < n)
        src.append(np.stack([ids[ok], rr[ok] * n + cc[ok]], 1))
    # advertisement order per node: right, left, up, down
    allp = np.concatenate(src)
    kind = np.concatenate([np.full(len(s), k) for k, s in enumerate(src)])
    o = np.lexsort((kind, allp[:, 0]))
    s_, d_ = allp[o, 0], allp[o, 1]
    if weighted_seed is None:
        met = np.ones(s_.size, np.int64)
    else:
        met = np.random.default_rng(weighted_seed).integers(1, max_metric + 1, s_.size)
    names = [str(i) for i in range(n * n)]
    return _stream_from_edges(names, ids + 1, s_, d_, met, 100001 + d_)


def fabric_names(pods: int, planes: int, ssw_per_plane: int = SSW_PER_PLANE,
                 rsw_per_pod: int = RSW_PER_POD) -> Tuple[List[str], Dict[str, np.ndarray]]:
    ssw = [f"1-{p}-{i}" for p in range(planes) for i in range(ssw_per_plane)]
    fsw = [f"2-{d}-{p}" for d in range(pods) for p in range(planes)]
    rsw = [f"3-{d}-{i}" for d in range(pods) for i in range(rsw_per_pod)]
    return ssw + fsw + rsw, dict(n_ssw=len(ssw), n_fsw=len(fsw), n_rsw=len(rsw))


def fabric(pods: int, planes: int = 8, ssw_per_plane: int = SSW_PER_PLANE,
           rsw_per_pod: int = RSW_PER_POD, reference_quirk: bool = False,
           weighted_seed: Optional[int] = None, max_metric: int = 64) -> AdjDbStream:
    """SSW/FSW/RSW fabric (createFabric). Ingest order: SSWs, FSWs, RSWs."""
    names, meta = fabric_names(pods, planes, ssw_per_plane, rsw_per_pod)
    nS, nF = meta["n_ssw"], meta["n_fsw"]
    S = lambda p, i: p * ssw_per_plane + i                      # noqa: E731
    F = lambda d, p: nS + d * planes + p                        # noqa: E731
    R = lambda d, i: nS + nF + d * rsw_per_pod + i              # noqa: E731
    P, D = np.meshgrid(np.arange(planes), np.arange(pods), indexing="ij")
    chunks_s, chunks_d, chunks_lbl = [], [], []
    # SSW (plane p, i): one FSW (pod d, plane p) per pod, pod-major order
    pp, ii, dd = np.meshgrid(np.arange(planes), np.arange(ssw_per_plane),
                             np.arange(pods if not reference_quirk else 1), indexing="ij")
    chunks_s.append(S(pp, ii).ravel())
    chunks_d.append(F(dd, pp).ravel())
    chunks_lbl.append((FSW * 100000 + dd * 100 + pp).ravel())
    # FSW (pod d, plane p): SSWs of plane p, then RSWs of pod d
    dd, pp, ii = np.meshgrid(np.arange(pods), np.arange(planes), np.arange(ssw_per_plane),
                             indexing="ij")
    fs_src, fs_dst = F(dd, pp), S(pp, ii)
    fs_lbl = SSW * 100000 + pp * 100 + ii
    dd2, pp2, jj = np.meshgrid(np.arange(pods), np.arange(planes), np.arange(rsw_per_pod),
                               indexing="ij")
    fr_src, fr_dst = F(dd2, pp2), R(dd2, jj)
    fr_lbl = RSW * 100000 + dd2 * 100 + jj
    # interleave per FSW: its SSW block then its RSW block
    fsrc = np.concatenate([fs_src.reshape(-1, ssw_per_plane), fr_src.reshape(-1, rsw_per_pod)], 1)
    fdst = np.concatenate([fs_dst.reshape(-1, ssw_per_plane), fr_dst.reshape(-1, rsw_per_pod)], 1)
    flbl = np.concatenate([fs_lbl.reshape(-1, ssw_per_plane), fr_lbl.reshape(-1, rsw_per_pod)], 1)
    chunks_s.append(fsrc.ravel())
    chunks_d.append(fdst.ravel())
    chunks_lbl.append(flbl.ravel())
    # RSW (pod d, i): FSWs of pod d
    dd, ii, pp = np.meshgrid(np.arange(pods), np.arange(rsw_per_pod), np.arange(planes),
                             indexing="ij")
    chunks_s.append(R(dd, ii).ravel())
    chunks_d.append(F(dd, pp).ravel())
    chunks_lbl.append((FSW * 100000 + dd * 100 + pp).ravel())
    src = np.concatenate(chunks_s).astype(np.int64)
    dst = np.concatenate(chunks_d).astype(np.int64)
    lbl = np.concatenate(chunks_lbl).astype(np.int64)
    if reference_quirk:
        # FSWs of pods > 0 still advertise their SSWs, but the SSW side only
        # advertises pod 0, so those adjacencies never form links. Keep them
        # (they are one-sided) by dropping them from the reverse-edge check:
        keep = np.ones(src.size, bool)
        is_f = (src >= nS) & (src < nS + nF) & (dst < nS)
        keep &= ~(is_f & (((src - nS) // planes) > 0))
        onesided = np.nonzero(~keep)[0]
        src_k, dst_k, lbl_k = src[keep], dst[keep], lbl[keep]
    else:
        src_k, dst_k, lbl_k = src, dst, lbl
    if weighted_seed is None:
        met = np.ones(src_k.size, np.int64)
    else:
        met = np.random.default_rng(weighted_seed).integers(1, max_metric + 1, src_k.size)
    labels = np.arange(len(names)) + 1
    st = _stream_from_edges(names, labels, src_k, dst_k, met, lbl_k)
    if reference_quirk:
        st = _add_one_sided(st, names, src[onesided], dst[onesided])
    return st


def _add_one_sided(st: AdjDbStream, names, src, dst) -> AdjDbStream:
    dbs = st.to_dbs()
    by = {db.name: db for db in dbs}
    for a, b in zip(src.tolist(), dst.tolist()):
        by[names[a]].adjs.append(create_adjacency(names[b], f"if_{names[a]}_{names[b]}",
                                                  f"if_{names[b]}_{names[a]}"))
    return AdjDbStream.from_dbs(dbs)


def hilbert_index(x: np.ndarray, y: np.ndarray, order: int) -> np.ndarray:
    """Position of integer points (0 <= x, y < 2**order) along a Hilbert curve."""
    n = 1 << order
    x = x.astype(np.int64).copy()
    y = y.astype(np.int64).copy()
    d = np.zeros_like(x)
    s = n >> 1
    while s > 0:
        rx = (x & s) > 0
        ry = (y & s) > 0
        d += s * s * ((3 * rx.astype(np.int64)) ^ ry.astype(np.int64))
        flip = ~ry & rx
        x = np.where(flip, n - 1 - x, x)
        y = np.where(flip, n - 1 - y, y)
        x, y = np.where(~ry, y, x), np.where(~ry, x, y)
        s >>= 1
    return d


def mesh(n_points: int, seed: int = 42, mean_degree: float = 8.0) -> AdjDbStream:
    """Random geometric mesh (largest component), metric in [1, 16] (SURVEY.md
    §8d M1M). Node names m%07d follow a Hilbert curve over the square, so
    spatially near nodes get near names and near node ids (the engine's id =
    name rank): a shortest-path wavefront then walks through nearby memory.
    The reference leaves the naming of this synthetic topology open."""
    rng = np.random.default_rng(seed)
    pts = rng.random((n_points, 2))
    r = float(np.sqrt(mean_degree / (np.pi * n_points)))
    cells = int(np.floor(1.0 / r))
    cx = np.minimum((pts[:, 0] * cells).astype(np.int64), cells - 1)
    cy = np.minimum((pts[:, 1] * cells).astype(np.int64), cells - 1)
    cell = cx * cells + cy
    order = np.argsort(cell, kind="stable")
    cstart = np.searchsorted(cell[order], np.arange(cells * cells + 1))
    srcs, dsts = [], []
    for dx in (-1, 0, 1):
        for dy in (-1, 0, 1):
            nx, ny = cx + dx, cy + dy
            ok = (nx >= 0) & (nx < cells) & (ny >= 0) & (ny < cells)
            idx = np.nonzero(ok)[0]
            nc = nx[idx] * cells + ny[idx]
            lo, hi = cstart[nc], cstart[nc + 1]
            cnt = hi - lo
            rep = np.repeat(idx, cnt)
            offs = np.arange(cnt.sum()) - np.repeat(np.cumsum(cnt) - cnt, cnt)
            cand = order[np.repeat(lo, cnt) + offs]
            m = rep < cand
            srcs.append(rep[m])
            dsts.append(cand[m])
    a = np.concatenate(srcs)
    b = np.concatenate(dsts)
    d = np.hypot(*(pts[a] - pts[b]).T)
    keep = d <= r
    a, b, d = a[keep], b[keep], d[keep]
    # largest connected component (union-find)
    from scipy.sparse import coo_matrix
    from scipy.sparse.csgraph import connected_components
    _, comp = connected_components(
        coo_matrix((np.ones(a.size, np.int8), (a, b)), shape=(n_points, n_points)),
        directed=False)
    alive = comp == np.bincount(comp).argmax()
    newid = -np.ones(n_points, np.int64)
    keep_idx = np.nonzero(alive)[0]
    q = np.minimum((pts[keep_idx] * 1024).astype(np.int64), 1023)
    newid[keep_idx[np.argsort(hilbert_index(q[:, 0], q[:, 1], 10), kind="stable")]] = \
        np.arange(keep_idx.size)
    m = alive[a]
    a, b, d = newid[a[m]], newid[b[m]], d[m]
    rtt = 100.0 + 1500.0 * d / r
    met = np.maximum(1, np.floor(rtt / 100.0)).astype(np.int64)
    V = int(alive.sum())
    src = np.concatenate([a, b])
    dst = np.concatenate([b, a])
    mm = np.concatenate([met, met])
    o = np.lexsort((dst, src))
    names = [f"m{i:07d}" for i in range(V)]
    return _stream_from_edges(names, np.arange(V) + 1, src[o], dst[o], mm[o],
                              np.zeros(src.size, np.int64))


def from_adjmap(adjmap: Sequence[Tuple[int, Sequence[Tuple[int, int]]]],
                db_order: Optional[Sequence[int]] = None) -> AdjDbStream:
    """DecisionTestUtils.cpp:15-45 ``getLinkState``: names ``"{n}"``, ifNames
    ``"{n}/{adj}/{k}"`` (k = parallel index), metric per entry, adjLabel
    (node<<16)+adj, nodeLabel = node. ``db_order`` gives the ingest order
    (the reference iterates an ``std::unordered_map<int,...>``; see
    tests/golden/make_golden.py for how that order is reproduced)."""
    entries = dict(adjmap)
    keys = list(db_order) if db_order is not None else [k for k, _ in adjmap]
    dbs = []
    for node in keys:
        par: Dict[int, int] = {}
        adjs = []
        for item in entries[node]:
            other, metric = (item, 1) if isinstance(item, int) else item
            k = par.get(other, 0)
            par[other] = k + 1
            adjs.append(create_adjacency(str(other), f"{node}/{other}/{k}",
                                         f"{other}/{node}/{k}", metric, (node << 16) + other))
        dbs.append(AdjDb(str(node), adjs, node))
    return AdjDbStream.from_dbs(dbs)
