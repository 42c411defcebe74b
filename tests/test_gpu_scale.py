"""Parity at BASELINE.json's full sizes: F10k all-sources,
F100k KSP2 + per-neighbour LFA runs from "2-0-0", and M1M sampled roots, each
against the CPU oracle, plus size-independent properties over every run the
oracle cannot afford (reached counts, twin-run equality, edge-disjoint KSP2
paths whose cost equals the SPF distance, and per-edge triangle / tight-
predecessor checks on whole distance rows)."""
import time

import numpy as np
import pytest

from oracle import Oracle
from openr_amd import topology as T
from openr_amd.engine import Engine
from openr_amd.linkstate import LinkState

pytestmark = pytest.mark.gpu


T0 = time.time()


def note(msg):
    """progress to stdout (run with -s): long CPU-side stages stay visible"""
    print(f"[{time.time() - T0:7.1f}s] {msg}", flush=True)


def both(stream):
    o, p = Oracle(), LinkState()
    assert o.apply(stream) == p.apply(stream)
    note("ingested")
    return o, p


@pytest.mark.timeout(600)
def test_f10k_all_sources_digests_and_properties():
    st = T.fabric(pods=173, planes=8)
    o, p = both(st)
    names = p.node_names()
    V = len(names)
    got = p.digests(names)
    note("F10k GPU digests")
    # every root against the CPU restatement (CSR Dijkstra, unit metric)
    assert np.array_equal(got, o.fast_digests(names, True, threads=16))
    # properties: connected fabric, no drains -> every run reaches V; a twin
    # run in reverse root order (different batches / classes) is identical
    assert np.all(got[:, 0] == V)
    assert np.array_equal(p.digests(names[::-1])[::-1], got)
    # full SpfResult text (next hops + pathLinks) for one root of each role
    for r in ("1-3-17", "2-100-5", "3-172-47"):
        assert p.spf_text(r) == o.spf_text(r)


def _path_cost(p, path, src):
    cost, at = 0, src
    for key in path:
        a, b = key.split("|")
        na, nb = a.split("%", 1)[0], b.split("%", 1)[0]
        nxt = nb if na == at else na
        cost += next(m for k, m, _ in p.links(at) if k == key)
        at = nxt
    return cost, at


@pytest.mark.timeout(900)
def test_f100k_ksp2_and_lfa_from_fsw():
    st = T.fabric(pods=1781, planes=8)
    o, p = both(st)
    src = "2-0-0"
    # spines of this and other planes, far pods' FSWs and RSWs, a local RSW
    dsts = ["1-0-35", "1-3-17", "1-7-0", "2-1780-5", "2-900-0", "3-1780-0", "3-900-47", "3-0-0"]
    assert p.ksp2_text(src, dsts) == o.ksp2_text(src, dsts)
    note("F100k KSP2 text equal")
    spf = p.spf(src)
    for d in dsts:
        k1, k2 = p.kth_paths(src, d, 1), p.kth_paths(src, d, 2)
        assert k1, d
        used = {key for path in k1 for key in path}
        for path in k1:
            cost, end = _path_cost(p, path, src)
            assert end == d and cost == spf[d][0], (d, path)
        for path in k2:
            assert not used & set(path), (d, path)  # edge-disjoint from k = 1
            cost, end = _path_cost(p, path, src)
            assert end == d and cost >= spf[d][0]
    # LFA: one SPF per neighbour of the source (its 48 RSWs and 36 spines)
    nbrs = sorted({k.split("|")[0].split("%")[0] if not k.startswith(src + "%") else
                   k.split("|")[1].split("%")[0] for k, _, _ in p.links(src)})
    assert len(nbrs) == 48 + 36
    assert np.array_equal(p.digests(nbrs), o.fast_digests(nbrs, True, threads=16))


def _role_stratified(names, k=256, extra=("1-3-5", "1-7-35", "3-900-17")):
    """scripts/bench_ksp2.py's parity sample: a quarter spines spread over
    every plane, 3/8 fabric switches, the rest racks (seed 0x5eed), + extras"""
    rng = np.random.default_rng(0x5EED)
    role = np.array([int(nm.split("-")[0]) for nm in names])
    pick = []
    for r_, share in ((1, k // 4), (2, (3 * k) // 8), (3, k - k // 4 - (3 * k) // 8)):
        cand = np.nonzero(role == r_)[0]
        pick.extend(int(x) for x in rng.choice(cand, min(share, cand.size), replace=False))
    out = sorted(set(pick))
    idx = {nm: i for i, nm in enumerate(names)}
    out += [idx[x] for x in extra if idx[x] not in out]
    return [names[i] for i in out]


@pytest.mark.timeout(900)
def test_f100k_ksp2_role_stratified_vs_oracle():
    """BASELINE config 4 at full size: KSP2 (k = 1 and k = 2 paths, text)
    from "2-0-0" to 259 role-stratified destinations through
    odl::LinkState (device KSP2, decremental k = 2 reruns) == the oracle's
    reference-shaped getKthPaths; then every destination's records from the
    decremental reruns == those of the full masked reruns (engine level)."""
    from openr_amd import _native as N
    st = T.fabric(pods=1781, planes=8)
    o, p = both(st)
    names = p.node_names()
    src = "2-0-0"
    sn = _role_stratified(names)
    assert len(sn) == 259
    got = p.ksp2_text(src, sn)
    note("F100k KSP2 259 destinations on the GPU")
    want = o.ksp2_text(src, sn, threads=16)
    note("oracle KSP2")
    assert got == want
    eng = Engine(0)
    eng.load(p.csr())
    try:
        s = names.index(src)
        dsts = list(range(len(names)))
        s0 = eng.ksp2_stats()
        k1, k2, stt = eng.ksp2(s, dsts, path_cap=1024)
        s1 = eng.ksp2_stats()
        import os
        os.environ["OSPF_KSP_NODECR"] = "1"
        try:
            f1, f2, fst = eng.ksp2(s, dsts, path_cap=1024)
        finally:
            del os.environ["OSPF_KSP_NODECR"]
        assert np.array_equal(stt, fst)
        assert k1 == f1 and k2 == f2
        took = s1["decremental"] - s0["decremental"]
        reruns = int(np.count_nonzero(stt & N.OSPF_KSP_RERUN))
        note(f"decremental {took} of {reruns} reruns, "
             f"{(s1['affected'] - s0['affected']) / max(1, took):.1f} affected nodes per run")
        assert took > 0.5 * reruns
    finally:
        eng.close()


@pytest.mark.timeout(900)
def test_m1m_sampled_roots_and_triangle_checks():
    st = T.mesh(1_000_000, seed=42)
    o, p = both(st)
    names = p.node_names()
    V = len(names)
    rng = np.random.default_rng(0x5eed)
    ids = rng.choice(V, 64, replace=False)
    roots = [names[i] for i in ids]
    dig = p.digests(roots)
    note("M1M GPU digests")
    assert np.array_equal(dig[:2], o.fast_digests(roots[:2], True, threads=2))
    csr = p.csr()
    e = Engine()
    try:
        e.load(csr)
        rows = e.run(ids, max(e.nh_words(int(i)) for i in ids), want_nh=False)["dist"]
    finally:
        e.close()
    rp = csr["row_ptr"].astype(np.int64)
    src = np.repeat(np.arange(V), np.diff(rp))
    col, met = csr["col"].astype(np.int64), csr["metric"].astype(np.int64)
    up = csr["edge_up"].astype(bool)
    nt = csr["no_transit"].astype(bool)
    inf = np.uint32(0xFFFFFFFF)
    for k, r in enumerate(ids):
        d = rows[k].astype(np.int64)
        reached = rows[k] != inf
        assert reached.sum() == int(dig[k][0]) and d[reached].sum() == int(dig[k][1])
        relax = up & reached[src] & ((src == r) | ~nt[src])
        cand = d[src[relax]] + met[relax]
        # triangle: no relaxable edge improves a distance
        assert np.all(d[col[relax]] <= cand)
        # every reached node but the root has a tight predecessor
        tight = np.zeros(V, bool)
        tight[col[relax][d[col[relax]] == cand]] = True
        assert np.all(tight[reached] | (np.arange(V)[reached] == r))


@pytest.mark.timeout(900)
def test_f100k_all_sources_sweep_role_stratified():
    """The headline path at full size: the F100k
    all-sources sweep (derive: ospf_levels_dev + ospf_nh_derive_dev behind
    ospf_sweep_run) against the CSR-Dijkstra restatement on EVERY spine (288,
    56-word rows), 256 fabric switches and 256 racks; reached == V for every
    root; and derive == the per-batch engine path bit for bit -- digests of a
    1,000-root sample across the three classes, whole dist + next-hop rows of
    8 roots per class."""
    from openr_amd.engine import Sweep
    st = T.fabric(pods=1781, planes=8)
    o, p = both(st)
    names = p.node_names()
    V = len(names)
    csr = p.csr()
    eng = Engine()
    eng.load(csr)
    sw = Sweep(eng)
    assert sw.mode == "derive"
    sw.run()
    eng.sync()
    d = np.zeros((V, 3), np.uint64)
    sw._check(sw._L.ospf_sweep_digests_host(sw._h, d.ctypes.data))
    got = np.zeros_like(d)
    got[sw.roots] = d
    note("F100k sweep digests")
    assert np.all(got[:, 0] == V)  # connected, no drains: every run reaches V
    role = np.array([int(n.split("-")[0]) for n in names])
    rng = np.random.default_rng(0x5EED)
    spines = np.nonzero(role == 1)[0]
    fsw = np.sort(rng.choice(np.nonzero(role == 2)[0], 256, replace=False))
    rsw = np.sort(rng.choice(np.nonzero(role == 3)[0], 256, replace=False))
    assert spines.size == 288
    strat = np.concatenate([spines, fsw, rsw])
    want = o.fast_digests([names[i] for i in strat], True, threads=16)
    note("F100k CSR-Dijkstra digests of the stratified set")
    bad = [names[r] for j, r in enumerate(strat) if not np.array_equal(got[r], want[j])]
    assert not bad, bad[:8]
    # derive == batch on a 1,000-root sample (100 spines, 300 FSWs, 600 RSWs)
    pick = {1: np.sort(rng.choice(spines, 100, replace=False)),
            2: np.sort(rng.choice(np.nonzero(role == 2)[0], 300, replace=False)),
            3: np.sort(rng.choice(np.nonzero(role == 3)[0], 600, replace=False))}
    for k, grp in pick.items():
        W = max(eng.nh_words(int(r)) for r in grp)
        ref = eng.run(grp, W, want_dist=False, want_nh=False, want_digest=True)["digest"]
        assert np.array_equal(got[grp], ref), k
        few = grp[:8]
        rows = eng.run(few, W)
        dist, nh = sw.rows(few, W)
        assert np.array_equal(dist, rows["dist"]), k
        assert np.array_equal(nh, rows["nh"]), k
    note("F100k derive == batch")
    sw.close()
    eng.close()


@pytest.mark.timeout(900)
def test_f100k_sweep_whole_rows_vs_reference_runspf():
    """Whole rows at full size against an independent restatement (VERDICT
    r04 weak #2: the other whole-row checks compare the sweep with the same
    engine's batch path): LinkState's all-sources sweep (prefetch_all: the
    sweep's dist + next-hop rows behind getSpfResult) against the oracle's
    reference-shaped runSpf (openr/decision/LinkState.cpp:836-911) as text --
    every node's metric and next-hop set -- for spines, fabric switches and
    racks, link metric and hop count."""
    st = T.fabric(pods=1781, planes=8)
    o, p = both(st)
    p.prefetch_all()
    p.prefetch_all(False)
    assert p.sweep_stats()["sweeps"] >= 1
    note("F100k sweeps")
    for r in ["1-3-17", "2-0-0", "2-900-5", "3-0-0", "3-1000-47", "3-1780-13"]:
        assert p.spf_text(r) == o.spf_text(r), r
    for r in ["1-7-35", "2-1780-7", "3-421-9"]:
        assert p.spf_text(r, False) == o.spf_text(r, False), r
    note("F100k whole rows vs the reference-shaped runSpf")
