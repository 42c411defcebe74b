"""GPU parity: the MI355X engine (through the C ABI) vs the CPU oracle and the
reference's own fixtures. Bit-exact: integer distances, next-hop name sets,
pathLinks order, KSP2 paths, digests. Run with ``-m gpu`` on an MI355X."""
import os

import numpy as np
import pytest

from golden_eval import ProductLS, load_fixtures, run_fixture
from graphs import random_stream
from oracle import Oracle, parse_spf_text
from openr_amd import topology as T
from openr_amd.adjdb import AdjDb, AdjDbStream, create_adjacency
from openr_amd import _native as N
from openr_amd.engine import Engine, EngineError
from openr_amd.linkstate import LinkState

pytestmark = pytest.mark.gpu

FIXTURES = load_fixtures()


@pytest.fixture(params=["auto", "0", "1", "2", "4", "5", "6", "7"])
def variant(request, monkeypatch):
    """Run each parity test with the planner's choice and with every other
    kernel variant forced where its state fits (OSPF_FORCE_VARIANT): 0/1/2 =
    Dial kernel (LDS / mixed / HBM state), 3/4 = BFS kernel (LDS bitmaps,
    byte next-hops in LDS / next-hops in HBM; unit metric only), 5 =
    multi-source bit-parallel BFS (unit metric, no ignored links), 6 =
    bucketed Dial (frontier lists; any metric <= 63), 7 = wave-per-root
    bucketed Dial (any metric, per-run ignored links)."""
    if request.param == "auto":
        monkeypatch.delenv("OSPF_FORCE_VARIANT", raising=False)
    else:
        monkeypatch.setenv("OSPF_FORCE_VARIANT", request.param)
    return request.param


@pytest.mark.parametrize("fx", FIXTURES, ids=[f["name"] for f in FIXTURES])
def test_reference_fixture_on_gpu(fx, variant):
    assert run_fixture(fx, ProductLS) > 0


def both(stream):
    o, p = Oracle(), LinkState()
    assert o.apply(stream) == p.apply(stream)
    return o, p


@pytest.mark.parametrize("seed", range(8))
@pytest.mark.parametrize("unit", [False, True])
def test_random_graph_all_roots_spf_text(seed, unit, variant):
    st, names = random_stream(seed, unit=unit)
    o, p = both(st)
    p.prefetch(names)  # one batched engine launch for every root
    for r in names:
        assert p.spf_text(r) == o.spf_text(r), r
        assert p.spf_text(r, False) == o.spf_text(r, False), r


@pytest.mark.parametrize("seed", range(4))
@pytest.mark.parametrize("unit", [False, True])
def test_random_graph_ksp2_batch(seed, unit, variant):
    st, names = random_stream(100 + seed, n=30, p=0.25, unit=unit)
    o, p = both(st)
    for src in names[:5]:
        assert p.ksp2_text(src, names) == o.ksp2_text(src, names), src
    assert p.spf_runs == o.spf_runs


KSP_KNOBS = {
    "default": {},
    "rows": {"OSPF_KSP_ROWS": "1"},          # per-run reruns + trace over dist rows
    "deep": {"OSPF_KSP_D0": "2"},            # level continuation past the first launch
    "one_batch_rounds": {"OSPF_MS_NB": "1"},  # one 64-run batch per round
    "tiny_records": {"ODL_KSP_CAP": "6"},     # record overflow -> host path per destination
    "heavy": {"OSPF_KSP_BUDGET": "3"},        # most runs resumed by the 16-wave kernel
    "no_heavy": {"OSPF_KSP_NOHEAVY": "1"},    # single-wave DFS only
    "no_decr": {"OSPF_KSP_NODECR": "1"},      # every k = 2 run by the full masked reruns
}


@pytest.mark.parametrize("knob", list(KSP_KNOBS), ids=list(KSP_KNOBS))
@pytest.mark.parametrize("unit", [True, False])
@pytest.mark.parametrize("seed", range(3))
def test_ksp2_device_trace_matches_oracle(seed, unit, knob, monkeypatch):
    """Device KSP2 (ospf_ksp2_run: k = 1 trace, masked reruns, k = 2 trace)
    through LinkState.prefetchKsp2, every destination of 90-node graphs with
    parallel links, down links and overloaded nodes (several 64-run batches)."""
    for k, v in KSP_KNOBS[knob].items():
        monkeypatch.setenv(k, v)
    st, names = random_stream(300 + seed, n=90, p=0.06, unit=unit)
    o, p = both(st)
    for src in names[:3]:
        assert p.ksp2_text(src, names) == o.ksp2_text(src, names), src
    assert p.spf_runs == o.spf_runs


@pytest.mark.parametrize("budget", ["default", "3"])
def test_fabric_ksp2_from_fsw_all_destinations(budget, monkeypatch):
    """BASELINE config 4 shape (KSP2 from FSW "2-0-0" to every node), small;
    budget 3 resumes nearly every trace on the 16-wave kernel."""
    if budget != "default":
        monkeypatch.setenv("OSPF_KSP_BUDGET", budget)
    st = T.fabric(pods=8, planes=4)
    o, p = both(st)
    dsts = p.node_names()
    assert p.ksp2_text("2-0-0", dsts) == o.ksp2_text("2-0-0", dsts)
    assert p.spf_runs == o.spf_runs


@pytest.mark.parametrize("unit", [True, False])
@pytest.mark.parametrize("seed", range(4))
def test_ksp2_decremental_equals_full_reruns(seed, unit, monkeypatch):
    """The k = 2 masked reruns by decremental SSSP (ospf_ksp2: lost tight
    supports from the source's row, fused trace) give every destination the
    same records and status words as the full masked reruns (OSPF_KSP_NODECR;
    itself oracle-pinned above), and the decremental kernel takes runs: random
    graphs with parallel / down links and overloaded nodes, and a drained
    fabric whose destinations include every role."""
    from graphs import drained_fabric
    for st in (random_stream(700 + seed, n=120, p=0.05, unit=unit)[0],
               drained_fabric(10, 4, seed=seed, drain=0.04, down=0.03,
                              weighted_seed=None if unit else seed + 1)):
        p, csr = _csr_of(st)
        names = p.node_names()
        V = len(names)
        eng = Engine(0)
        eng.load(csr)
        try:
            for src in (0, V // 3, V - 1):
                dsts = list(range(V))
                s0 = eng.ksp2_stats()
                k1, k2, stt = eng.ksp2(src, dsts, path_cap=512)
                s1 = eng.ksp2_stats()
                monkeypatch.setenv("OSPF_KSP_NODECR", "1")
                f1, f2, fst = eng.ksp2(src, dsts, path_cap=512)
                monkeypatch.delenv("OSPF_KSP_NODECR")
                assert k1 == f1 and k2 == f2, src
                assert np.array_equal(stt, fst), src
                reruns = int(np.count_nonzero(stt & N.OSPF_KSP_RERUN))
                took = s1["decremental"] - s0["decremental"]
                sent = s1["full_reruns"] - s0["full_reruns"]
                assert took + sent == reruns, (took, sent, reruns)
                # unit metric: ECMP DAGs, small affected sets; weighted SPF
                # DAGs are near-trees, where a cut link takes its subtree
                # (those runs may all take the full reruns)
                assert not unit or reruns == 0 or took > 0, (took, sent, reruns)
        finally:
            eng.close()


def test_engine_ksp2_budget_status():
    """Records that do not fit path_cap come back flagged, not truncated."""
    p, csr = _csr_of(T.fabric(pods=3, planes=2))
    eng = Engine(0)
    eng.load(csr)
    names = p.node_names()
    src = names.index("2-0-0")
    k1, k2, st = eng.ksp2(src, list(range(len(names))), path_cap=512)
    assert all(x is not None for x in k1) and all(x is not None for x in k2)
    assert k1[src] == [] and k2[src] == []
    assert all(len(k1[d]) >= 1 for d in range(len(names)) if d != src)
    # every k = 1 path starts at src's links and is edge-disjoint from the others
    for d in range(len(names)):
        flat = [l for path in k1[d] for l in path]
        assert len(flat) == len(set(flat))
    k1s, k2s, sts = eng.ksp2(src, list(range(len(names))), path_cap=2)
    for d in range(len(names)):
        if d == src:
            assert k1s[d] == [] and sts[d] == 0
        else:
            assert k1s[d] is None and k2s[d] is None and sts[d] & 0x2


def test_unknown_and_isolated_roots():
    st, names = random_stream(7)
    extra = AdjDbStream.from_dbs([AdjDb("zz-isolated", [], 99)])
    o, p = both(st)
    assert o.apply(extra) == p.apply(extra)
    for r in ("zz-isolated", "not-a-node"):
        assert p.spf_text(r) == o.spf_text(r)
        assert p.kth_paths(r, names[0], 2) == o.kth_paths(r, names[0], 2)


def test_incremental_updates_keep_parity():
    """Topology changes invalidate the memo and the device snapshot
    (LinkState.cpp:721-724); non-topology updates keep the memo."""
    st, names = random_stream(21, n=30)
    o, p = both(st)
    rng = np.random.default_rng(5)
    dbs = st.to_dbs()
    for step in range(6):
        db = dbs[int(rng.integers(len(dbs)))]
        if step % 3 == 0:
            db.overloaded = not db.overloaded
        elif step % 3 == 1 and db.adjs:
            a = db.adjs[int(rng.integers(len(db.adjs)))]
            a.metric = int(rng.integers(1, 30))
        else:
            db.node_label += 1000
        upd = AdjDbStream.from_dbs([db])
        assert o.apply(upd) == p.apply(upd)
        for r in names[:8]:
            assert p.spf_text(r) == o.spf_text(r)
    assert p.spf_runs == o.spf_runs


@pytest.mark.parametrize("seed", range(3))
def test_default_mode_events_patch_in_place(seed):
    """Default (non-incremental) mode: metric, link up / down and overload
    events on the same nodes and links are patched into the CSR and the
    device graph in place (no re-snapshot), the memo is still
    dropped on every topology change and kept on label-only updates
    (LinkState.cpp:721-724, 751-754): link-metric and hop-count results,
    KSP2 paths and decision.spf_runs equal the oracle's after every event."""
    st, names = random_stream(700 + seed, n=36)
    o, p = both(st)
    rng = np.random.default_rng(seed)
    dbs = st.to_dbs()
    for step in range(12):
        db = dbs[int(rng.integers(len(dbs)))]
        kind = step % 4
        if kind == 0:
            db.overloaded = not db.overloaded
        elif kind == 1 and db.adjs:
            a = db.adjs[int(rng.integers(len(db.adjs)))]
            a.metric = int(rng.integers(1, 40))
        elif kind == 2 and db.adjs:
            a = db.adjs[int(rng.integers(len(db.adjs)))]
            a.overloaded = not a.overloaded
        else:
            db.node_label += 7
        upd = AdjDbStream.from_dbs([db])
        assert o.apply(upd) == p.apply(upd)
        for r in names[:6]:
            assert p.spf_text(r) == o.spf_text(r), (step, r)
            assert p.spf_text(r, False) == o.spf_text(r, False), (step, r)
        a_, b_ = names[int(rng.integers(len(names)))], names[int(rng.integers(len(names)))]
        for k in (1, 2):
            assert p.kth_paths(a_, b_, k) == o.kth_paths(a_, b_, k), (step, a_, b_, k)
        assert p.spf_runs == o.spf_runs, step


def test_grid31_all_sources_digests():
    st = T.grid(31)
    o, p = both(st)
    roots = [str(i) for i in range(31 * 31)]
    assert np.array_equal(p.digests(roots), o.digests(roots, threads=8))
    # Manhattan distance sum check from the reference grid fixture semantics
    d = p.digests(["0"])[0]
    assert int(d[0]) == 961 and int(d[1]) == sum(r + c for r in range(31) for c in range(31))


def test_grid31_hop_count_and_weighted():
    st = T.grid(31, weighted_seed=3)
    o, p = both(st)
    roots = [str(i) for i in range(0, 961, 7)]
    assert np.array_equal(p.digests(roots), o.digests(roots, threads=8))
    assert np.array_equal(p.digests(roots, False), o.digests(roots, False, threads=8))


@pytest.mark.parametrize("weighted", [False, True])
def test_fabric_sampled_digests(weighted, variant):
    st = T.fabric(pods=12, planes=8, weighted_seed=7 if weighted else None)
    o, p = both(st)
    names = p.node_names()
    rng = np.random.default_rng(0x5eed)
    roots = [names[i] for i in rng.choice(len(names), 24, replace=False)]
    roots += ["1-0-0", "2-0-0", "3-0-0"]  # one SSW, FSW, RSW
    assert np.array_equal(p.digests(roots), o.digests(roots, threads=8))
    for r in roots[-3:]:
        assert p.spf_text(r) == o.spf_text(r)


@pytest.mark.parametrize("variant_env", [None, "2"])
def test_wide_root_nexthop_slices(variant_env, monkeypatch):
    """A spine with 140 distinct neighbours needs 5 next-hop words: the BFS
    kernel splits the row into 4-word slices run by separate workgroups."""
    if variant_env:
        monkeypatch.setenv("OSPF_FORCE_VARIANT", variant_env)
    st = T.fabric(pods=140, planes=2)
    o, p = both(st)
    roots = ["1-0-0", "1-1-35", "2-7-1", "3-139-47"]
    assert np.array_equal(p.digests(roots), o.digests(roots, threads=8))
    for r in roots:
        assert p.spf_text(r) == o.spf_text(r)
        assert p.spf_text(r, False) == o.spf_text(r, False)


def test_fabric_reference_quirk():
    st = T.fabric(pods=6, planes=4, reference_quirk=True)
    o, p = both(st)
    for r in ("1-0-0", "2-3-1", "3-5-7"):
        assert p.spf_text(r) == o.spf_text(r)


def test_mesh_sampled_digests():
    st = T.mesh(3000, seed=42)
    o, p = both(st)
    names = p.node_names()
    rng = np.random.default_rng(0x5eed)
    roots = [names[i] for i in rng.choice(len(names), 16, replace=False)]
    assert np.array_equal(p.digests(roots), o.digests(roots, threads=8))


@pytest.mark.parametrize("seed", range(4))
@pytest.mark.parametrize("unit", [False, True])
def test_incremental_linkstate_matches_full_recompute(seed, unit):
    """Incremental mode: metric / link up-down / node overload updates keep the
    memoised results of unaffected roots and patch the device graph in place;
    every root's result must equal the oracle's full recompute."""
    st, names = random_stream(500 + seed, n=40, unit=unit)
    o, p = both(st)
    p.set_incremental(True)
    p.prefetch(names)
    p.prefetch(names, False)
    rng = np.random.default_rng(seed)
    dbs = st.to_dbs()
    for step in range(9):
        db = dbs[int(rng.integers(len(dbs)))]
        kind = step % 3
        if kind == 0:
            db.overloaded = not db.overloaded
        elif db.adjs:
            a = db.adjs[int(rng.integers(len(db.adjs)))]
            if kind == 1 and not unit:
                a.metric = int(rng.integers(1, 30))
            else:
                a.overloaded = not a.overloaded  # link down / up
        upd = AdjDbStream.from_dbs([db])
        assert o.apply(upd) == p.apply(upd)
        for r in names:
            assert p.spf_text(r) == o.spf_text(r), (step, r)
            assert p.spf_text(r, False) == o.spf_text(r, False), (step, r)
    stats = p.incremental_stats()
    assert stats["patches"] > 0 and stats["kept"] > 0, stats


def test_engine_affected_roots_and_patch():
    """ospf_update_links patches the resident graph like a reload, and every
    run ospf_affected_roots leaves unflagged is bit-identical after the change."""
    import torch
    st, names = random_stream(77, n=70, p=0.08)
    p = LinkState(stream=st)
    csr = p.csr()
    V = len(names)
    eng = Engine(0)
    eng.load(csr)
    W = int(max(eng.nh_words(r) for r in range(V)))
    roots = np.arange(V, dtype=np.uint32)
    before = eng.run(roots, W)
    rp, col, lid = csr["row_ptr"], csr["col"], csr["link_id"]
    owner = np.repeat(np.arange(V), np.diff(rp.astype(np.int64)))
    rng = np.random.default_rng(3)
    new = {k: v.copy() for k, v in csr.items()}
    ups, changes = [], []
    for l in rng.choice(int(lid.max()) + 1, 4, replace=False):
        e = np.nonzero(lid == l)[0]
        lo, hi = (e[0], e[1]) if owner[e[0]] <= owner[e[1]] else (e[1], e[0])
        up0 = int(csr["edge_up"][lo])
        up1 = 1 - up0 if rng.random() < 0.4 else 1
        m_lo, m_hi = int(rng.integers(1, 21)), int(rng.integers(1, 21))
        new["edge_up"][[lo, hi]] = up1
        new["metric"][lo], new["metric"][hi] = m_lo, m_hi
        ups.append((int(l), up1, m_lo, m_hi))
        changes.append((0, int(owner[lo]), int(owner[hi]), up0, int(csr["metric"][lo]),
                        int(csr["metric"][hi]), up1, m_lo, m_hi))
    d_dist = torch.from_numpy(before["dist"].view(np.int32)).cuda()
    flags = torch.zeros(V, dtype=torch.uint8, device="cuda")
    eng.update_links(ups, version=2)
    eng.affected(d_dist.data_ptr(), V, changes, flags.data_ptr())
    eng.sync()
    after = eng.run(roots, W)
    fresh = Engine(0)
    fresh.load(new)
    ref = fresh.run(roots, W)
    assert np.array_equal(after["dist"], ref["dist"]) and np.array_equal(after["nh"], ref["nh"])
    f = flags.cpu().numpy().astype(bool)
    keep = ~f
    assert keep.any() and f.any()
    assert np.array_equal(after["dist"][keep], before["dist"][keep])
    assert np.array_equal(after["nh"][keep], before["nh"][keep])
    # in-place repair: every run it keeps (status 0) equals the fresh run
    d_nh = torch.from_numpy(before["nh"].view(np.int32)).cuda()
    st = torch.zeros(V, dtype=torch.int32, device="cuda")
    d_roots = torch.from_numpy(roots.view(np.int32)).cuda()
    eng.repair(d_roots.data_ptr(), V, W, d_dist.data_ptr(), d_nh.data_ptr(), changes,
               st.data_ptr())
    eng.sync()
    ok = st.cpu().numpy() == 0
    assert ok.any()
    rd = d_dist.cpu().numpy().view(np.uint32)
    rn = d_nh.cpu().numpy().view(np.uint32)
    assert np.array_equal(rd[ok], ref["dist"][ok]) and np.array_equal(rn[ok], ref["nh"][ok])


@pytest.mark.parametrize("seed", range(6))
def test_engine_repair_fabric_link_events(seed):
    """Link events in an ECMP fabric (unit metric): uplink down / up, metric
    change; repaired rows (status 0) equal fresh runs, most runs repair."""
    import torch
    p = LinkState(stream=T.fabric(pods=6, planes=4))
    csr = p.csr()
    V = p.num_nodes()
    eng = Engine(0)
    eng.load(csr)
    W = int(max(eng.nh_words(r) for r in range(V)))
    roots = np.arange(V, dtype=np.uint32)
    before = eng.run(roots, W)
    rp, lid = csr["row_ptr"], csr["link_id"]
    owner = np.repeat(np.arange(V), np.diff(rp.astype(np.int64)))
    rng = np.random.default_rng(seed)
    l = int(rng.integers(int(lid.max()) + 1))
    e = np.nonzero(lid == l)[0]
    lo, hi = (e[0], e[1]) if owner[e[0]] <= owner[e[1]] else (e[1], e[0])
    up1, m1 = (0, 1) if seed % 2 == 0 else (1, 3)
    ch = [(0, int(owner[lo]), int(owner[hi]), 1, 1, 1, up1, m1, m1)]
    eng.update_links([(l, up1, m1, m1)], version=2)
    d_roots = torch.from_numpy(roots.view(np.int32)).cuda()
    d_dist = torch.from_numpy(before["dist"].view(np.int32)).cuda()
    d_nh = torch.from_numpy(before["nh"].view(np.int32)).cuda()
    st = torch.zeros(V, dtype=torch.int32, device="cuda")
    eng.repair(d_roots.data_ptr(), V, W, d_dist.data_ptr(), d_nh.data_ptr(), ch, st.data_ptr())
    eng.sync()
    ref = eng.run(roots, W)
    ok = st.cpu().numpy() == 0
    rd = d_dist.cpu().numpy().view(np.uint32)
    rn = d_nh.cpu().numpy().view(np.uint32)
    assert np.array_equal(rd[ok], ref["dist"][ok]) and np.array_equal(rn[ok], ref["nh"][ok])
    if up1 == 0:
        assert ok.mean() > 0.5, ok.mean()


@pytest.mark.parametrize("forced", [None, "6"])
def test_mesh_60k_bucketed_dial_digests(forced, monkeypatch):
    """Weighted mesh too large for LDS state: the planner's wave-per-root Dial
    (variant 7) and the workgroup-per-root bucketed Dial (variant 6) against
    the oracle, sampled roots, digests (dist + next hops)."""
    if forced:
        monkeypatch.setenv("OSPF_FORCE_VARIANT", forced)
    st = T.mesh(60000, seed=7)
    o, p = both(st)
    names = p.node_names()
    rng = np.random.default_rng(11)
    roots = [names[i] for i in rng.choice(len(names), 12, replace=False)]
    eng = Engine(0)
    eng.load(p.csr())
    assert eng.plan(1)["variant"] == int(forced or 7)
    assert np.array_equal(p.digests(roots), o.digests(roots, threads=8))
    for r in roots[:2]:
        assert p.spf_text(r) == o.spf_text(r)


def test_fabric_ksp2_batch_from_rsw():
    st = T.fabric(pods=6, planes=4)
    o, p = both(st)
    dsts = p.node_names()[::7]
    assert p.ksp2_text("3-0-0", dsts) == o.ksp2_text("3-0-0", dsts)
    assert p.spf_runs == o.spf_runs


# ------------------------------------------------------------ engine ABI
def _csr_of(stream):
    p = LinkState(stream=stream)
    return p, p.csr()


def test_engine_direct_batch_matches_linkstate():
    p, csr = _csr_of(T.grid(12))
    eng = Engine(0)
    eng.load(csr)
    roots = np.arange(144, dtype=np.uint32)
    out = eng.run(roots, 1, want_digest=True)
    names = p.node_names()
    assert np.array_equal(out["digest"], p.digests(names))
    # dist from node "0" in a 12x12 grid is the Manhattan distance (ids are
    # name ranks: "0" < "1" < "10" < ...)
    root0 = names.index("0")
    r, c = np.divmod(np.array([int(n) for n in names]), 12)
    assert np.array_equal(out["dist"][root0], (r + c).astype(np.uint32))
    assert eng.spf_runs == 144


def test_engine_rejects_out_of_contract():
    p, csr = _csr_of(T.grid(4))
    eng = Engine(0)
    bad = dict(csr)
    bad["metric"] = csr["metric"].copy()
    bad["metric"][0] = 0
    with pytest.raises(EngineError) as ei:
        eng.load(bad)
    assert ei.value.code == -4
    eng.load(csr)
    p2, csr2 = _csr_of(T.fabric(pods=2, planes=4))
    eng.load(csr2)
    ssw = p2.node_id("1-0-0")
    with pytest.raises(EngineError):  # nh_words too small for a root
        eng.run([ssw], 0)


def test_engine_device_api_and_error_word():
    torch = pytest.importorskip("torch")
    p, csr = _csr_of(T.fabric(pods=40, planes=8))
    eng = Engine(0)
    eng.load(csr)
    V = eng.V
    names = p.node_names()
    rsw = [p.node_id(f"3-{i}-0") for i in range(16)]
    d_roots = torch.tensor(rsw, dtype=torch.int32, device="cuda")
    d_dig = torch.zeros((16, 3), dtype=torch.int64, device="cuda")
    d_dist = torch.zeros((16, V), dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    eng.run_dev(d_roots.data_ptr(), 16, 1, flags=0x2 | 0x8, d_dist=d_dist.data_ptr(),
                d_digest=d_dig.data_ptr(), stream=s)
    eng.sync(s)
    want = p.digests([names[i] for i in rsw])
    assert np.array_equal(d_dig.cpu().numpy().view(np.uint64), want)
    ssw = torch.tensor([p.node_id("1-0-0")], dtype=torch.int32, device="cuda")
    eng.run_dev(ssw.data_ptr(), 1, 1, flags=0x8, d_digest=d_dig.data_ptr(), stream=s)
    with pytest.raises(EngineError):
        eng.sync(s)


# ------------------------------------------------ multi-source BFS (variant 5)
def _engine_for(stream):
    p = LinkState(stream=stream)
    eng = Engine(0)
    eng.load(p.csr())
    return p, eng


def _run_forced(eng, monkeypatch, variant, roots, W, **kw):
    monkeypatch.setenv("OSPF_FORCE_VARIANT", variant)
    return eng.run(roots, W, want_digest=True, **kw)


@pytest.mark.parametrize("seed", range(3))
@pytest.mark.parametrize("hop", [False, True])
@pytest.mark.parametrize("defer", [True, False])
def test_msbfs_matches_per_root_bfs(seed, hop, defer, monkeypatch):
    """Variant 5 (64 roots per traversal) vs variant 4 (one root per
    workgroup) on random unit graphs with parallel links, down links and
    overloaded nodes; 150 roots = two full 64-root batches + a ragged one.
    defer: rows written once at the end from per-(node, root) level bytes
    (default) or per level (OSPF_MS_NODEFER)."""
    if not defer:
        monkeypatch.setenv("OSPF_MS_NODEFER", "1")
    st, names = random_stream(300 + seed, n=150, p=0.05, unit=not hop)
    p, eng = _engine_for(st)
    roots = np.arange(eng.V, dtype=np.uint32)
    W = int(max(eng.nh_words(int(r)) for r in roots))
    a = _run_forced(eng, monkeypatch, "5", roots, W, hop_count=hop)
    b = _run_forced(eng, monkeypatch, "4", roots, W, hop_count=hop)
    assert np.array_equal(a["dist"], b["dist"])
    assert np.array_equal(a["nh"], b["nh"])
    assert np.array_equal(a["digest"], b["digest"])
    o = Oracle(st)
    assert np.array_equal(a["digest"], o.digests([p.node_names()[i] for i in roots],
                                                 not hop, threads=8))


@pytest.mark.parametrize("nb,R,ilv", [("1", None, 1), ("3", None, 1), ("8", None, 1), ("32", "3", 1),
                                      ("4", "7", 1), ("32", "20", 1), ("2", "1", 1),
                                      ("8", None, 0), ("32", "20", 0)])
def test_msbfs_wide_roots_and_rounds(nb, R, ilv, monkeypatch):
    """Spines with 140 distinct neighbours need 5 next-hop words = 5 passes
    per 64-root batch; OSPF_MS_NB bounds the (batch, pass) pairs per round so
    the sweep spans several rounds; nh_words above the need is zero-filled.
    OSPF_MS_R packs the bit-planes: R roots per batch, 64/R planes per word,
    64/R next-hop words per pass. ilv: multi-word rows staged word-major and
    interleaved (OSPF_MS_ILV=1) or stored word by word from each pass
    (OSPF_MS_ILV=0; the default below 8 words)."""
    monkeypatch.setenv("OSPF_MS_NB", nb)
    monkeypatch.setenv("OSPF_MS_ILV", str(ilv))
    if R:
        monkeypatch.setenv("OSPF_MS_R", R)
    st = T.fabric(pods=140, planes=2)
    p, eng = _engine_for(st)
    names = p.node_names()
    rng = np.random.default_rng(1)
    roots = np.concatenate([[p.node_id(n) for n in ("1-0-0", "1-1-35", "2-7-1", "3-139-47")],
                            rng.choice(eng.V, 90, replace=False)]).astype(np.uint32)
    a = _run_forced(eng, monkeypatch, "5", roots, 6)
    b = _run_forced(eng, monkeypatch, "4", roots, 6)
    assert np.array_equal(a["dist"], b["dist"])
    assert np.array_equal(a["nh"], b["nh"])
    o = Oracle(st)
    assert np.array_equal(a["digest"], o.digests([names[i] for i in roots], threads=8))


def test_msbfs_device_api_hint_and_error_word():
    """ospf_run_batch_dev with max_root_neighbors: rack switches (8
    neighbours) run with 8 bit-planes; a spine under the same hint raises the
    device error word."""
    torch = pytest.importorskip("torch")
    p, eng = _engine_for(T.fabric(pods=40, planes=8))
    V = eng.V
    names = p.node_names()
    rsw = [p.node_id(f"3-{i}-{j}") for i in range(40) for j in range(2)]
    n = len(rsw)
    assert eng.plan(1, 0x2 | 0x4, n_roots=n, max_root_neighbors=8)["variant"] == 5
    d_roots = torch.tensor(rsw, dtype=torch.int32, device="cuda")
    d_dig = torch.zeros((n, 3), dtype=torch.int64, device="cuda")
    d_dist = torch.zeros((n, V), dtype=torch.int32, device="cuda")
    d_nh = torch.zeros((n, V, 1), dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    eng.run_dev(d_roots.data_ptr(), n, 1, flags=0x2 | 0x4 | 0x8, d_dist=d_dist.data_ptr(),
                d_nh=d_nh.data_ptr(), d_digest=d_dig.data_ptr(), stream=s, max_root_neighbors=8)
    eng.sync(s)
    want = p.digests([names[i] for i in rsw])
    assert np.array_equal(d_dig.cpu().numpy().view(np.uint64), want)
    ref = eng.run(np.array(rsw, np.uint32), 1)
    assert np.array_equal(d_dist.cpu().numpy().view(np.uint32), ref["dist"])
    assert np.array_equal(d_nh.cpu().numpy().view(np.uint32), ref["nh"])
    bad = torch.tensor(rsw[:40] + [p.node_id("2-0-0")], dtype=torch.int32, device="cuda")
    eng.run_dev(bad.data_ptr(), 41, 4, flags=0x8, d_digest=d_dig.data_ptr(), stream=s,
                max_root_neighbors=8)
    with pytest.raises(EngineError):
        eng.sync(s)


# ------------------------------------------------ UCMP
@pytest.mark.parametrize("seed", range(4))
@pytest.mark.parametrize("algo", ["adj", "prefix"])
def test_ucmp_random_graphs_match_oracle(seed, algo):
    """resolveUcmpWeights over the GPU SPF result vs the oracle's restatement
    (LinkState.cpp:913-1033): leaves = every node at one distance from the
    root, random weights; also a leaf set at mixed distances (skipped: empty)."""
    st, names = random_stream(500 + seed, n=40, p=0.12)
    o, p = both(st)
    rng = np.random.default_rng(seed)
    for root in names[:6]:
        spf = p.spf(root)
        by_d = {}
        for n, (m, _, _) in spf.items():
            if n != root:
                by_d.setdefault(m, []).append(n)
        if not by_d:
            continue
        d = sorted(by_d)[len(by_d) // 2]
        leaves = {n: int(rng.integers(1, 9)) for n in by_d[d]}
        assert p.ucmp(root, leaves, algo) == o.ucmp(root, leaves, algo)
        if len(by_d) > 1:
            mixed = {by_d[sorted(by_d)[0]][0]: 1, by_d[sorted(by_d)[-1]][0]: 1}
            assert p.ucmp(root, mixed, algo) == o.ucmp(root, mixed, algo) == {}


@pytest.mark.parametrize("case", ["overload", "unoverload", "link_down", "metric"])
def test_engine_repair_wide_and_node_events(case):
    """Repair with spine roots wider than 8 next-hop words (300 pods: W = 10)
    and with overload toggles; repaired rows (status 0) equal fresh runs."""
    import torch
    p = LinkState(stream=T.fabric(pods=300, planes=2, ssw_per_plane=4, rsw_per_pod=4))
    csr = p.csr()
    names = p.node_names()
    V = p.num_nodes()
    eng = Engine(0)
    eng.load(csr)
    W = int(max(eng.nh_words(r) for r in range(V)))
    assert W >= 10
    roots = np.arange(V, dtype=np.uint32)
    rp, lid = csr["row_ptr"], csr["link_id"]
    owner = np.repeat(np.arange(V), np.diff(rp.astype(np.int64)))
    fsw = names.index("2-17-1")
    if case == "unoverload":
        eng.update_nodes([fsw], [1], version=2)
    before = eng.run(roots, W)
    if case in ("overload", "unoverload"):
        eng.update_nodes([fsw], [1 if case == "overload" else 0], version=3)
        ch = [(1, fsw, 0, 0, 0, 0, 0, 0, 0)]
    else:
        rsw = names.index("3-42-2")
        e = next(int(e) for e in range(rp[rsw], rp[rsw + 1]) if csr["col"][e] == names.index("2-42-0"))
        l = int(lid[e])
        ee = np.nonzero(lid == l)[0]
        lo, hi = (ee[0], ee[1]) if owner[ee[0]] <= owner[ee[1]] else (ee[1], ee[0])
        up1, m1 = (0, 1) if case == "link_down" else (1, 2)
        ch = [(0, int(owner[lo]), int(owner[hi]), 1, 1, 1, up1, m1, m1)]
        eng.update_links([(l, up1, m1, m1)], version=3)
    d_roots = torch.from_numpy(roots.view(np.int32)).cuda()
    d_dist = torch.from_numpy(before["dist"].view(np.int32)).cuda()
    d_nh = torch.from_numpy(before["nh"].view(np.int32)).cuda()
    st = torch.zeros(V, dtype=torch.int32, device="cuda")
    eng.repair(d_roots.data_ptr(), V, W, d_dist.data_ptr(), d_nh.data_ptr(), ch, st.data_ptr())
    eng.sync()
    ref = eng.run(roots, W)
    ok = st.cpu().numpy() == 0
    rd = d_dist.cpu().numpy().view(np.uint32)
    rn = d_nh.cpu().numpy().view(np.uint32)
    assert np.array_equal(rd[ok], ref["dist"][ok]) and np.array_equal(rn[ok], ref["nh"][ok])
    spines = np.array([n.startswith("1-") for n in names])
    assert ok.mean() > 0.3, ok.mean()
    assert (ok & spines).any()  # wide rows repaired too


# ------------------------------------------ wave-per-root Dial (variant 7)
WD_KNOBS = {
    "default": {},
    "tagged": {"OSPF_WD_DELTA": "3"},                      # buckets of 3 distances
    "overflow": {"OSPF_WD_BCAP": "4"},                     # lists overflow -> node scans
    "tagged_overflow": {"OSPF_WD_DELTA": "5", "OSPF_WD_BCAP": "3"},
    "wave": {"OSPF_WD_GROUP": "1"},                        # a wave per root
    "cu": {"OSPF_WD_GROUP": "16"},                         # a 16-wave group per root
    "unpacked": {"OSPF_WD_PACK": "0"},                     # dist / next-hop rows as state
    "pack16": {"OSPF_WD_PACK": "16"},                      # 16-bit next-hop field
}


@pytest.mark.parametrize("knob", list(WD_KNOBS), ids=list(WD_KNOBS))
@pytest.mark.parametrize("wmax", [20, 200, 100000])
@pytest.mark.parametrize("seed", range(3))
def test_wdial_random_graphs_any_metric(seed, wmax, knob, monkeypatch):
    """Variant 7 on random graphs with parallel, down and overloaded links and
    metrics up to 200 (ring of one list per distance) and 100,000 (buckets of
    several distances with tagged entries); full SPF text of every root, in
    link-metric and hop-count mode, against the oracle."""
    monkeypatch.setenv("OSPF_FORCE_VARIANT", "7")
    for k, v in WD_KNOBS[knob].items():
        monkeypatch.setenv(k, v)
    st, names = random_stream(900 + seed, n=60, p=0.1, wmax=wmax)
    o, p = both(st)
    p.prefetch(names)
    for r in names:
        assert p.spf_text(r) == o.spf_text(r), r
        assert p.spf_text(r, False) == o.spf_text(r, False), r


@pytest.mark.parametrize("knob", ["default", "tagged", "overflow"])
def test_wdial_ksp2_reruns_with_ignored_links(knob, monkeypatch):
    """KSP2 masked reruns through variant 7 (per-run ignore lists read from
    HBM) on a weighted graph with metrics above 63."""
    monkeypatch.setenv("OSPF_FORCE_VARIANT", "7")
    for k, v in WD_KNOBS[knob].items():
        monkeypatch.setenv(k, v)
    st, names = random_stream(950, n=40, p=0.15, wmax=500)
    o, p = both(st)
    for src in names[:4]:
        assert p.ksp2_text(src, names) == o.ksp2_text(src, names), src
    assert p.spf_runs == o.spf_runs


@pytest.mark.parametrize("max_metric", [64, 1000, 70000])
def test_weighted_fabric_metric_above_63(max_metric):
    """Weighted fabric (pods = 800, 45k nodes) with metrics 1..max_metric: the
    planner's large-graph weighted path (variant 7: state beyond LDS) vs the
    oracle's CSR-Dijkstra restatement (the reference-shaped heap needs ~2 min
    per root here), sampled roots of every switch class, in link-metric and
    hop-count mode."""
    st = T.fabric(pods=800, planes=8, weighted_seed=7, max_metric=max_metric)
    o, p = both(st)
    eng = Engine(0)
    eng.load(p.csr())
    assert eng.plan(1)["variant"] == 7
    names = p.node_names()
    rng = np.random.default_rng(0x5eed)
    roots = [names[i] for i in rng.choice(len(names), 60, replace=False)]
    roots += ["1-0-0", "1-7-35", "2-0-0", "3-0-0"]
    assert np.array_equal(p.digests(roots), o.fast_digests(roots, threads=8))
    assert np.array_equal(p.digests(roots, False), o.fast_digests(roots, False, threads=8))


def _chain_dbs(names, down):
    """A unit-metric chain; `down`: the middle link (19, 20) is drained."""
    out = []
    for i, nm in enumerate(names):
        adjs = []
        for j in (i - 1, i + 1):
            if 0 <= j < len(names):
                ov = down and i == 19 and j == 20
                adjs.append(create_adjacency(names[j], f"{nm}-{names[j]}", f"{names[j]}-{nm}", 1,
                                             overloaded=ov))
        out.append(AdjDb(nm, adjs, i + 1))
    return out


def test_depth_bound_after_bridge_drain_and_undrain():
    """draining a bridge recomputes the multi-source BFS
    level bound on the two halves (ids chosen so each half's seed sits in its
    middle: bound 22); undraining must recompute it again (the chain's hop
    diameter is 39), or roots past level 22 come back unreached. Incremental
    LinkState (the device graph patched in place), every root batched."""
    names = [("a" if i in (10, 30) else "m") + f"{i:02d}" for i in range(40)]
    o, p = Oracle(), LinkState()
    st = AdjDbStream.from_dbs(_chain_dbs(names, False))
    assert o.apply(st) == p.apply(st)
    p.set_incremental(True)
    for down in (True, False, True, False):
        upd = AdjDbStream.from_dbs([d for d in _chain_dbs(names, down)
                                    if d.name in (names[19], names[20])])
        assert o.apply(upd) == p.apply(upd)
        p.prefetch(names)
        for r in names:
            assert p.spf_text(r) == o.spf_text(r), (down, r)


def test_engine_depth_bound_link_up_recomputes():
    """Same at the C ABI: ospf_update_links down then up, the multi-source
    BFS over every root equals a fresh load of the same graph."""
    names = [("a" if i in (10, 30) else "m") + f"{i:02d}" for i in range(40)]
    lsx = LinkState(stream=AdjDbStream.from_dbs(_chain_dbs(names, False)))
    csr = lsx.csr()
    eng = Engine(0)
    eng.load(csr)
    V = eng.V
    i19, i20 = lsx.node_id(names[19]), lsx.node_id(names[20])
    rp, col, lid = csr["row_ptr"], csr["col"], csr["link_id"]
    e = next(e for e in range(rp[i19], rp[i19 + 1]) if col[e] == i20)
    roots = np.arange(V, dtype=np.uint32)
    for up in (0, 1):
        eng.update_links([(int(lid[e]), up, 1, 1)], version=2 + up)
        got = eng.run(roots, 1)
        ref_csr = {k: v.copy() for k, v in csr.items()}
        ref_csr["edge_up"][lid == lid[e]] = up
        fresh = Engine(0)
        fresh.load(ref_csr)
        want = fresh.run(roots, 1)
        assert np.array_equal(got["dist"], want["dist"]) and np.array_equal(got["nh"], want["nh"])
    assert int(got["dist"][lsx.node_id(names[0]), lsx.node_id(names[39])]) == 39


def test_engine_update_links_rejects_whole_batch():
    """a batch with one bad entry (unknown link id, or
    metric 0 on an up link) is rejected before any state changes: the graph,
    its unit-metric flag and the results stay those of before the call."""
    p, csr = _csr_of(T.fabric(pods=4, planes=2))
    eng = Engine(0)
    eng.load(csr)
    V = eng.V
    roots = np.arange(V, dtype=np.uint32)
    W = int(max(eng.nh_words(r) for r in range(V)))
    before = eng.run(roots, W)
    l0 = int(csr["link_id"][0])
    for bad in ([(l0, 1, 7, 7), (10 ** 6, 1, 1, 1)], [(l0, 0, 1, 1), (l0 + 1, 1, 0, 5)]):
        with pytest.raises(EngineError):
            eng.update_links(bad, version=9)
        assert eng.info().unit_metric == 1
        after = eng.run(roots, W)
        assert np.array_equal(after["dist"], before["dist"])
        assert np.array_equal(after["nh"], before["nh"])


@pytest.mark.parametrize("pack", ["8", "16"])
def test_wdial_packed_overflow_falls_back(pack, monkeypatch):
    """Packed state (dist << K | next hops) with distances that outgrow the
    field (metrics up to 100,000 on a long chain: > 2^24) aborts the packed
    run and reruns the root unpacked: same rows as the unpacked kernel."""
    monkeypatch.setenv("OSPF_FORCE_VARIANT", "7")
    names = [f"c{i:03d}" for i in range(300)]
    dbs = []
    for i, nm in enumerate(names):
        adjs = [create_adjacency(names[j], f"{nm}-{names[j]}", f"{names[j]}-{nm}", 90000 + j)
                for j in (i - 1, i + 1) if 0 <= j < len(names)]
        dbs.append(AdjDb(nm, adjs, i + 1))
    st = AdjDbStream.from_dbs(dbs)
    o, p = both(st)
    eng = Engine(0)
    eng.load(p.csr())
    roots = np.arange(eng.V, dtype=np.uint32)
    monkeypatch.setenv("OSPF_WD_PACK", pack)
    a = eng.run(roots, 1, want_digest=True)
    monkeypatch.setenv("OSPF_WD_PACK", "0")
    b = eng.run(roots, 1, want_digest=True)
    assert int(a["dist"].max()) > (1 << 24)
    assert np.array_equal(a["dist"], b["dist"]) and np.array_equal(a["nh"], b["nh"])
    assert np.array_equal(a["digest"], o.fast_digests(names, threads=8))


def test_wdial_packed_edges_follow_link_updates(monkeypatch):
    """Variant 7 reads {colx, w | rw << 16} entries while every metric fits 16
    bits: ospf_update_links patches them with the separate arrays, and a
    metric above 0xFFFF drops them (the kernel reads the arrays). Each state
    equals a fresh load of the same graph."""
    monkeypatch.setenv("OSPF_FORCE_VARIANT", "7")
    st, names = random_stream(61, n=60, p=0.1, wmax=30)
    p = LinkState(stream=st)
    csr = p.csr()
    eng = Engine(0)
    eng.load(csr)
    V = eng.V
    roots = np.arange(V, dtype=np.uint32)
    W = int(max(eng.nh_words(r) for r in range(V)))
    rp, lid = csr["row_ptr"], csr["link_id"]
    owner = np.repeat(np.arange(V), np.diff(rp.astype(np.int64)))
    rng = np.random.default_rng(4)
    cur = {k: v.copy() for k, v in csr.items()}
    for step, big in enumerate([False, False, True, False]):
        ups = []
        for l in rng.choice(int(lid.max()) + 1, 5, replace=False):
            e = np.nonzero(lid == l)[0]
            lo, hi = (e[0], e[1]) if owner[e[0]] <= owner[e[1]] else (e[1], e[0])
            m_lo = int(rng.integers(1, 40)) + (100000 if big else 0)
            m_hi = int(rng.integers(1, 40))
            up = int(rng.random() > 0.2)
            cur["edge_up"][[lo, hi]] = up
            cur["metric"][lo], cur["metric"][hi] = m_lo, m_hi
            ups.append((int(l), up, m_lo, m_hi))
        eng.update_links(ups, version=2 + step)
        got = eng.run(roots, W)
        fresh = Engine(0)
        fresh.load({k: v.copy() for k, v in cur.items()})
        want = fresh.run(roots, W)
        assert np.array_equal(got["dist"], want["dist"]), step
        assert np.array_equal(got["nh"], want["nh"]), step


@pytest.mark.parametrize("nb", [None, "1", "7", "24"])
def test_msbfs_merged_rows_match_per_pass_rows(nb, monkeypatch):
    """Multi-pass batches (fabric switches: 84 neighbours = 3 next-hop words)
    write their rows with one kernel for all passes (msbfs_rows_multi) -- the
    same dist / next-hop rows and digests as the per-pass rows kernels
    (OSPF_MS_NOMERGE), at several round sizes (OSPF_MS_NB), and as the
    oracle's digests; a ragged last batch and nh_words above the need
    (zero-filled words) included."""
    if nb:
        monkeypatch.setenv("OSPF_MS_NB", nb)
    monkeypatch.setenv("OSPF_FORCE_VARIANT", "5")
    st = T.fabric(pods=40, planes=8)
    p, eng = _engine_for(st)
    names = p.node_names()
    fsw = np.array([p.node_id(n) for n in names if n.startswith("2-")], np.uint32)[:150]
    for W in (3, 5):
        a = eng.run(fsw, W, want_digest=True)
        monkeypatch.setenv("OSPF_MS_NOMERGE", "1")
        b = eng.run(fsw, W, want_digest=True)
        monkeypatch.delenv("OSPF_MS_NOMERGE")
        assert np.array_equal(a["dist"], b["dist"]) and np.array_equal(a["nh"], b["nh"]), W
        assert np.array_equal(a["digest"], b["digest"])
    o = Oracle(st)
    assert np.array_equal(a["digest"], o.digests([names[i] for i in fsw], threads=8))


@pytest.mark.parametrize("incremental", [False, True])
def test_out_of_contract_update_switches_to_host_and_back(incremental):
    """An update that puts a metric-0 / negative adjacency on a live graph moves
    its link-metric runs to the host path (incremental patching steps aside);
    hop-count runs stay on the engine; restoring the metric returns to it."""
    stream, names = random_stream(31, n=40)
    o, p = Oracle(), LinkState()
    p.set_incremental(incremental)
    assert o.apply(stream) == p.apply(stream)

    def check():
        for r in names:
            assert p.spf(r) == parse_spf_text(o.spf_text(r, True)), r
            assert p.spf(r, False) == parse_spf_text(o.spf_text(r, False)), r

    check()
    db = next(d for d in stream.to_dbs() if len(d.adjs) >= 2)
    orig = [a.metric for a in db.adjs]
    for metric in (0, -3):
        db.adjs[0].metric = metric
        db.adjs[1].metric = 0
        s = AdjDbStream.from_dbs([db])
        assert o.apply(s) == p.apply(s)
        check()
    for a, m in zip(db.adjs, orig):
        a.metric = m
    s = AdjDbStream.from_dbs([db])
    assert o.apply(s) == p.apply(s)
    check()


def test_ksp2_ignore_set_above_run_list_cap():
    """k = 2 with more k = 1 path links than one run's ignore list holds
    (OSPF_MAX_IGNORED_PER_RUN = 2048): 1,100 two-hop shortest paths s-m_i-d
    (2,200 links) plus a 3-hop detour; device KSP2 records overflow too."""
    n_mid = 1100
    dbs = {"s": [], "d": [], "a": [], "b": []}
    for i in range(n_mid):
        m = f"m{i:04d}"
        dbs[m] = [create_adjacency("s", f"{m}/s", f"s/{m}", 1),
                  create_adjacency("d", f"{m}/d", f"d/{m}", 1)]
        dbs["s"].append(create_adjacency(m, f"s/{m}", f"{m}/s", 1))
        dbs["d"].append(create_adjacency(m, f"d/{m}", f"{m}/d", 1))
    for x, y in (("s", "a"), ("a", "b"), ("b", "d")):
        dbs[x].append(create_adjacency(y, f"{x}/{y}", f"{y}/{x}", 1))
        dbs[y].append(create_adjacency(x, f"{y}/{x}", f"{x}/{y}", 1))
    stream = AdjDbStream.from_dbs(AdjDb(n, a, i + 1) for i, (n, a) in enumerate(dbs.items()))
    o, p = Oracle(), LinkState()
    assert o.apply(stream) == p.apply(stream)
    k1 = p.kth_paths("s", "d", 1)
    assert len(k1) == n_mid and sum(len(x) for x in k1) > 2048
    assert k1 == o.kth_paths("s", "d", 1)
    k2 = p.kth_paths("s", "d", 2)
    assert k2 == o.kth_paths("s", "d", 2) and len(k2) == 1 and len(k2[0]) == 3
    assert p.spf("s") == parse_spf_text(o.spf_text("s", True))  # graph restored
    q = LinkState()
    q.apply(stream)
    assert q.ksp2_text("s", ["d", "a"]) == o.ksp2_text("s", ["d", "a"])


def test_ksp2_ignore_overflow_repeated_keeps_metric_runs():
    """ADVICE r02 (link_state.cpp KSP2 path): a k = 2 run whose ignore set
    overflows one run's list masks those links on the device and restores them
    (ospf_links_mask / unmask) -- repeated calls must not ratchet the engine's
    distance bound: with metrics of 100,000 twelve calls would push a bound
    that grew by every restored link past 2^32, and later link-metric runs
    would fail. Every call and the runs after it equal the oracle."""
    n_mid, M = 1100, 100000
    dbs = {"s": [], "d": [], "a": [], "b": []}
    for i in range(n_mid):
        m = f"m{i:04d}"
        dbs[m] = [create_adjacency("s", f"{m}/s", f"s/{m}", M),
                  create_adjacency("d", f"{m}/d", f"d/{m}", M)]
        dbs["s"].append(create_adjacency(m, f"s/{m}", f"{m}/s", M))
        dbs["d"].append(create_adjacency(m, f"d/{m}", f"{m}/d", M))
    for x, y in (("s", "a"), ("a", "b"), ("b", "d")):
        dbs[x].append(create_adjacency(y, f"{x}/{y}", f"{y}/{x}", M))
        dbs[y].append(create_adjacency(x, f"{y}/{x}", f"{x}/{y}", M))
    stream = AdjDbStream.from_dbs(AdjDb(n, a, i + 1) for i, (n, a) in enumerate(dbs.items()))
    o, p = Oracle(), LinkState()
    assert o.apply(stream) == p.apply(stream)
    want2 = o.kth_paths("s", "d", 2)
    assert len(want2) == 1 and len(want2[0]) == 3
    for _ in range(12):
        assert p.kth_paths("s", "d", 2) == want2
    for root in ("s", "d", "a", "m0007"):
        assert p.spf(root) == parse_spf_text(o.spf_text(root, True)), root
