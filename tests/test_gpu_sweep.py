"""All-sources sweeps through the library (ospf_sweep_*, include/openr_spf.h):
every path the engine can take (derive, weighted cover, weighted derive,
batch) must give every root the rows and digest of the per-batch engine path
-- itself oracle-pinned -- bit for bit; the multi-device context
(ospf_multi_* / ospf_msweep_*) must partition the roots and gather the same
digests; odl::LinkState's all-sources entry points must use the sweep.
Reference semantics: LinkState::runSpf, openr/decision/LinkState.cpp:836-911;
the all-sources caller is Decision::getDecisionRouteDb per node
(openr/decision/Decision.cpp:309)."""
import numpy as np
import pytest

from graphs import drained_fabric, random_stream
from oracle import Oracle
from openr_amd import topology as T
from openr_amd.adjdb import AdjDb, AdjDbStream, create_adjacency
from openr_amd.engine import Engine, EngineError, Multi, MultiSweep, Sweep
from openr_amd.linkstate import LinkState

pytestmark = pytest.mark.gpu


def engine_for(stream):
    ls = LinkState()
    ls.apply(stream)
    csr = ls.csr()
    eng = Engine()
    eng.load(csr)
    return ls, csr, eng


def sweep_digests(sw):
    d = np.zeros((max(1, sw.n_roots), 3), np.uint64)
    sw._check(sw._L.ospf_sweep_digests_host(sw._h, d.ctypes.data))
    return dict(zip(sw.roots.tolist(), d[: sw.n_roots]))


def check_sweep_vs_batch(eng, mode="auto", hop=False, rows_for=None, hip_graph=True,
                         want_mode=None):
    """Every root's digest from the sweep == the batch path's; rows too for
    `rows_for` roots (all when None and the graph is small)."""
    V = eng.V
    sw = Sweep(eng, mode=mode, hop_count=hop, hip_graph=hip_graph)
    try:
        if want_mode:
            assert sw.mode == want_mode
        assert sorted(sw.roots.tolist()) == list(range(V))
        sw.run()
        eng.sync()
        got = sweep_digests(sw)
        words = np.array([eng.nh_words(r) for r in range(V)])
        for W in sorted(set(words.tolist())):
            grp = np.nonzero(words == W)[0].astype(np.uint32)
            ref = eng.run(grp, W, hop_count=hop, want_digest=True)
            for j, r in enumerate(grp.tolist()):
                assert np.array_equal(got[r], ref["digest"][j]), (mode, r)
            pick = grp if rows_for is None else np.intersect1d(grp, rows_for)
            if pick.size:
                idx = np.searchsorted(grp, pick)
                dist, nh = sw.rows(pick, W)
                assert np.array_equal(dist, ref["dist"][idx]), (mode, W)
                assert np.array_equal(nh, ref["nh"][idx]), (mode, W)
        return sw.mode
    finally:
        sw.close()


@pytest.mark.parametrize("seed", range(4))
def test_sweep_random_unit_graphs_every_mode(seed):
    stream, _ = random_stream(seed, n=70, unit=True)
    _, _, eng = engine_for(stream)
    try:
        assert check_sweep_vs_batch(eng, "auto") == "lds"  # a small graph: the LDS sweep
        for mode in ("derive", "wderive", "batch", "lds"):
            check_sweep_vs_batch(eng, mode)
        check_sweep_vs_batch(eng, "derive", hip_graph=False)
        check_sweep_vs_batch(eng, "lds", hip_graph=False)
        check_sweep_vs_batch(eng, "auto", hop=True)
        check_sweep_vs_batch(eng, "derive", hop=True)
    finally:
        eng.close()


@pytest.mark.parametrize("seed", range(4))
def test_sweep_random_weighted_graphs_every_mode(seed):
    stream, _ = random_stream(seed + 10, n=70, unit=False, wmax=50)
    _, _, eng = engine_for(stream)
    try:
        m = check_sweep_vs_batch(eng, "auto")
        assert m in ("wcover", "wderive")
        for mode in ("wderive", "batch"):
            check_sweep_vs_batch(eng, mode)
        try:
            check_sweep_vs_batch(eng, "wcover")
        except EngineError as e:  # outside the cover kernel's limits
            assert e.code == -4, e
        check_sweep_vs_batch(eng, "auto", hop=True)  # hop count: lds / derive on any metric
        check_sweep_vs_batch(eng, "lds", hop=True)
        with pytest.raises(EngineError):  # link metrics != 1: not the LDS kernel's contract
            Sweep(eng, mode="lds")
    finally:
        eng.close()


def test_sweep_fabric_with_drains_vs_oracle():
    """A fabric (3 width classes) with drained switches and down links: the
    derive sweep == batch path, and the digests == the CPU restatement."""
    st = drained_fabric(6, 4, seed=3)
    ls, csr, eng = engine_for(st)
    try:
        assert check_sweep_vs_batch(eng, "auto", rows_for=np.arange(0, eng.V, 7)) == "lds"
        check_sweep_vs_batch(eng, "derive", rows_for=np.arange(0, eng.V, 7))
        names = ls.node_names()
        want = Oracle(st).fast_digests(names)
        for mode in ("lds", "derive"):
            sw = Sweep(eng, mode=mode)
            sw.run()
            got = sweep_digests(sw)
            for r in range(eng.V):
                assert np.array_equal(got[r], want[r]), (mode, names[r])
            sw.close()
    finally:
        eng.close()


@pytest.mark.parametrize("hop", [False, True])
def test_sweep_early_start_equals_eager(hop):
    """OSPF_SWEEP_EARLY_START (the first run's serial prefix queued while the
    plan is built, odl::LinkState's re-sweep): digests and rows == a sweep
    created and run the plain way, on a drained fabric in derive mode."""
    st = drained_fabric(24, 4, seed=9)
    ls, csr, eng = engine_for(st)
    try:
        base = Sweep(eng, mode="derive", hop_count=hop)
        base.run()
        want = sweep_digests(base)
        base.close()
        def same(got):
            return sorted(got) == sorted(want) and all(np.array_equal(got[r], want[r]) for r in want)

        for _ in range(2):  # (the second: pooled blocks, streams and events)
            sw = Sweep(eng, mode="derive", hop_count=hop, hip_graph=False, defer=True,
                       early_start=True)
            sw.run()
            assert same(sweep_digests(sw))
            sw.run()  # a later run of the same sweep: the plain eager path
            assert same(sweep_digests(sw))
            sw.close()
    finally:
        eng.close()


def test_sweep_weighted_fabric_cover_path():
    st = T.fabric(pods=8, planes=4, weighted_seed=7)
    ls, csr, eng = engine_for(st)
    try:
        assert check_sweep_vs_batch(eng, "auto", rows_for=np.arange(0, eng.V, 5),
                                    want_mode="wcover") == "wcover"
        check_sweep_vs_batch(eng, "wderive", rows_for=np.arange(0, eng.V, 11))
    finally:
        eng.close()


@pytest.mark.parametrize("stage", [False, True, "tiled"])
@pytest.mark.parametrize("drain", [0.0, 0.08])
def test_sweep_weighted_fabric_closure(drain, stage, monkeypatch):
    """A weighted fabric whose cover splits into seeds (the spines) and small
    components (a pod's fabric switches): the closure path -- the seeds' Dial,
    closure_kernel's cover columns, then the full rows -- == the batch path bit
    for bit, with drained (overloaded) switches and down links."""
    # 40 pods: a spine has 40 > 32 neighbours, so it is no leaf candidate and
    # stays in the cover (as on F100k)
    if stage == "tiled":  # closure rows by node tiles x root chunks (opt-in)
        monkeypatch.setenv("OSPF_COVER_ROWS_TILED", "1")
    elif stage:  # closure rows in chunks, leaf chunks on a second stream (opt-in)
        monkeypatch.setenv("OSPF_WCOVER_STAGE", "1")
    st = drained_fabric(40, 4, seed=5, drain=drain, down=0.03 if drain else 0.0,
                        weighted_seed=11, ssw_per_plane=4)
    _, _, eng = engine_for(st)
    try:
        sw = Sweep(eng, mode="wcover")
        prof = sw.profile(1)
        sw.close()
        names = [p["name"] for p in prof]
        assert "cover_closure" in names and "cover_seeds" in names, names
        # the seeds' next hops come out of their Dial (masks at settle)
        seeds_k = [p.get("kernel", "") for p in prof if p["name"] == "cover_seeds"][0]
        assert "next-hop masks" in seeds_k, seeds_k
        rows_k = [p.get("kernel", "") for p in prof if p["name"].startswith("cover_rows")]
        assert ("closure_tile_rows_kernel" in rows_k[0]) == (stage == "tiled"), rows_k
        check_sweep_vs_batch(eng, "wcover", rows_for=np.arange(0, eng.V, 7))
    finally:
        eng.close()


@pytest.mark.parametrize("opt_in", ["seed", "derive", "opt_in"])
@pytest.mark.parametrize("drain", [0.0, 0.05])
def test_sweep_weighted_wide_cover_roots_runs(drain, opt_in, monkeypatch):
    """Spines with > 128 neighbours (W = 5 next-hop words) on the weighted
    cover path == the batch path bit for bit, with drained switches and down
    links: next hops by the seeds' Dial (masks at settle, the default), by
    the neighbour-row derivation (OSPF_SEED_NONH), and by the opt-in
    wnh_runs_kernel (runs of a plane's spines, lane = node, a wave per word)
    + wnh_hub_kernel (hub rows in LDS per tile) -- OSPF_WNH_RUNS / OSPF_WNH_HUB."""
    if opt_in != "seed":  # the neighbour-row kernels (no masks from the Dial / closure)
        monkeypatch.setenv("OSPF_SEED_NONH", "1")
        monkeypatch.setenv("OSPF_CLOSURE_NONH", "1")
    if opt_in == "opt_in":
        monkeypatch.setenv("OSPF_WNH_RUNS", "1")
        monkeypatch.setenv("OSPF_WNH_HUB", "1")
    st = drained_fabric(130, 2, seed=9, drain=drain, down=0.02 if drain else 0.0,
                        weighted_seed=3, ssw_per_plane=4)
    _, _, eng = engine_for(st)
    try:
        sw = Sweep(eng, mode="wcover")
        prof = sw.profile(1)
        sw.close()
        wide = [p for p in prof if p["name"].startswith("wderive_wide_w")]
        if opt_in == "seed":
            seeds_k = " ".join(p.get("kernel", "") for p in prof if p["name"] == "cover_seeds")
            assert "next-hop masks" in seeds_k, [p["name"] for p in prof]
        else:
            assert any(int(p["name"].rsplit("w", 1)[1]) > 4 for p in wide), [p["name"] for p in prof]
        if opt_in == "opt_in":
            kern = " ".join(p.get("kernel", "") for p in wide)
            assert "wnh_runs_kernel" in kern and "wnh_hub_kernel" in kern, kern
        check_sweep_vs_batch(eng, "wcover", rows_for=np.arange(0, eng.V, 13))
    finally:
        eng.close()


@pytest.mark.parametrize("seed", range(3))
def test_sweep_wmulti_random_graphs(seed):
    """The multi-root traversal (OSPF_SWEEP_WMULTI: groups of 32 roots share a
    wavefront, [node][root] distances) + derived leaf rows and next hops ==
    the batch path bit for bit: weighted random graphs with overloaded nodes,
    hop count, and a drained weighted fabric; parts of a partition too."""
    stream, _ = random_stream(seed + 40, n=90, unit=False, wmax=30)
    _, _, eng = engine_for(stream)
    try:
        check_sweep_vs_batch(eng, "wmulti", want_mode="wmulti")
        check_sweep_vs_batch(eng, "wmulti", hop=True, want_mode="wmulti")
        check_sweep_vs_batch(eng, "wmulti", hip_graph=False, want_mode="wmulti")
    finally:
        eng.close()


def test_sweep_wmulti_drained_fabric_and_mesh(monkeypatch):
    st = drained_fabric(12, 4, seed=6, drain=0.05, down=0.03, weighted_seed=5)
    _, _, eng = engine_for(st)
    try:
        check_sweep_vs_batch(eng, "wmulti", rows_for=np.arange(0, eng.V, 5), want_mode="wmulti")
        monkeypatch.setenv("OSPF_MSD_DELTA", "3")  # narrow buckets: more phases, same rows
        check_sweep_vs_batch(eng, "wmulti", rows_for=np.arange(0, eng.V, 9), want_mode="wmulti")
        monkeypatch.delenv("OSPF_MSD_DELTA")
    finally:
        eng.close()
    st = T.mesh(6000, seed=3)
    ls, csr, eng = engine_for(st)
    try:
        V = eng.V
        full = Sweep(eng, mode="wmulti")
        full.run()
        eng.sync()
        got = sweep_digests(full)
        full.close()
        names = ls.node_names()
        pick = list(range(0, V, 97)) + [V - 1]
        want = Oracle(st).fast_digests([names[i] for i in pick])
        for j, r in enumerate(pick):
            assert np.array_equal(got[r], want[j]), names[r]
        for n_parts in (3,):  # parts: every root once, same digests
            seen = {}
            for p in range(n_parts):
                sw = Sweep(eng, part=p, n_parts=n_parts, mode="wmulti")
                sw.run()
                eng.sync()
                seen.update(sweep_digests(sw))
                sw.close()
            assert sorted(seen) == list(range(V))
            for r in range(0, V, 13):
                assert np.array_equal(seen[r], got[r]), r
    finally:
        eng.close()


@pytest.mark.parametrize("delta", [None, "4"])
def test_sweep_wmulti_distances_near_2_32(delta, monkeypatch):
    """Distances up to 2^32 - 3 (metrics near 2^31, distance bound 2^32 - 2,
    the engine's limit): the multi-root traversal's bucket end is computed in
    64 bits and saturates, so the last bucket (whose end passes 2^32) drains
    instead of wrapping to a small end no deferred value reaches (ADVICE r04:
    spf_msdist.hip bucket end). Digests == the CSR-Dijkstra restatement."""
    if delta:
        monkeypatch.setenv("OSPF_MSD_DELTA", delta)
    big = 2 ** 31 - 1
    # a -> b -> c forward at ~2^31 each, back at 1; d hangs off c at 1 both ways
    spec = {"a": [("b", big)], "b": [("a", 1), ("c", big - 3)],
            "c": [("b", 1), ("d", 1)], "d": [("c", 1)]}
    # bound = big + (big - 3) + 1 + 1 = 2^32 - 4 < 2^32 - 1
    dbs = [AdjDb(n, [create_adjacency(m, f"{n}-{m}", f"{m}-{n}", w) for m, w in spec[n]], i + 1)
           for i, n in enumerate(sorted(spec))]
    st = AdjDbStream.from_dbs(dbs)
    ls, csr, eng = engine_for(st)
    try:
        sw = Sweep(eng, mode="wmulti", hip_graph=False)
        assert sw.mode == "wmulti"
        sw.run()
        eng.sync()
        got = sweep_digests(sw)
        sw.close()
        names = ls.node_names()
        want = Oracle(st).fast_digests(names)
        for r in range(eng.V):
            assert np.array_equal(got[r], want[r]), names[r]
    finally:
        eng.close()


def test_sweep_deep_unit_grid_does_not_raise():
    """Unit 100 x 100 grid: diameter 198, past derive's 123-level bound. AUTO
    must take another path and stay exact; sampled
    roots vs the CSR-Dijkstra restatement."""
    st = T.grid(100)
    ls, csr, eng = engine_for(st)
    try:
        sw = Sweep(eng)
        assert sw.mode != "derive"
        sw.run()
        eng.sync()
        got = sweep_digests(sw)
        assert len(got) == eng.V
        names = ls.node_names()
        pick = [0, 99, 4950, 5049, 9900, 9999] + list(range(101, 9999, 997))
        want = Oracle(st).fast_digests([names[i] for i in pick])
        for i, r in enumerate(pick):
            assert np.array_equal(got[r], want[i]), names[r]
        with pytest.raises(EngineError):
            Sweep(eng, mode="derive")
        sw.close()
    finally:
        eng.close()


@pytest.mark.parametrize("mode", ["derive", "lds"])
def test_sweep_poison_and_profile(mode):
    st = T.fabric(pods=4, planes=4)
    ls, csr, eng = engine_for(st)
    try:
        sw = Sweep(eng, mode=mode)
        sw.run()
        eng.sync()
        good = sweep_digests(sw)
        sw.poison()
        eng.sync()
        bad = sweep_digests(sw)
        assert all(np.all(v == np.uint64(0xFFFFFFFFFFFFFFFF)) for v in bad.values())
        sw.run()  # a replay rewrites every digest
        eng.sync()
        again = sweep_digests(sw)
        assert all(np.array_equal(good[r], again[r]) for r in good)
        prof = sw.profile(2)
        assert prof[0]["name"] == "levels" if mode == "derive" else prof[0]["name"].startswith("lds_w")
        assert all(p["ms_median"] > 0 and p["compulsory_bytes"] > 0 for p in prof)
        # a unit's bytes may include intermediate rows it writes for a later
        # unit (twin level rows when its dist rows are fused into the twin
        # next-hop unit); the step counts outputs only
        assert 0 < sw.step_compulsory_bytes <= sum(p["compulsory_bytes"] for p in prof)
        sw.close()
    finally:
        eng.close()


@pytest.mark.parametrize("mode", ["auto", "derive"])
def test_sweep_partition_parts_cover_every_root_once(mode):
    st = T.fabric(pods=9, planes=4)
    ls, csr, eng = engine_for(st)
    try:
        full = Sweep(eng, mode=mode)
        full.run()
        want = sweep_digests(full)
        full.close()
        seen = {}
        for n_parts in (2, 3):
            seen.clear()
            for p in range(n_parts):
                sw = Sweep(eng, part=p, n_parts=n_parts, mode=mode)
                sw.run()
                for r, d in sweep_digests(sw).items():
                    assert r not in seen
                    seen[r] = d
                # closure rows (+ the BFS'd leaf representatives of twin levels)
                assert sw.n_rows <= 1.6 * max(1, sw.n_roots) + 64 + (9 if mode == "derive" else 0)
                sw.close()
            assert len(seen) == eng.V
            assert all(np.array_equal(seen[r], want[r]) for r in range(eng.V))
    finally:
        eng.close()


def test_sweep_partition_weighted_closure():
    """Root-sharded weighted sweeps on the closure path (each part Dials every
    seed, closes only its own components' roots): 2 and 3 parts gather every
    root once with the full sweep's digests."""
    st = drained_fabric(40, 4, seed=6, drain=0.04, down=0.02, weighted_seed=13,
                        ssw_per_plane=4)
    _, _, eng = engine_for(st)
    try:
        full = Sweep(eng, mode="wcover")
        assert "cover_closure" in [p["name"] for p in full.profile(1)]
        full.run()
        want = sweep_digests(full)
        full.close()
        for n_parts in (2, 3):
            seen = {}
            for p in range(n_parts):
                sw = Sweep(eng, part=p, n_parts=n_parts, mode="wcover")
                sw.run()
                for r, d in sweep_digests(sw).items():
                    assert r not in seen
                    seen[r] = d
                sw.close()
            assert len(seen) == eng.V
            assert all(np.array_equal(seen[r], want[r]) for r in range(eng.V)), n_parts
    finally:
        eng.close()


@pytest.mark.parametrize("topo", ["unit", "weighted", "unit-derive"])
def test_multi_device_context_two_slots_on_device0(topo):
    """ospf_multi with two contexts on device 0: parts on each slot, digests
    gathered by peer copies (same-device copies here; RCCL / xGMI across
    devices is unexercised until a multi-GPU node runs it)."""
    st = T.fabric(pods=6, planes=4, weighted_seed=7 if topo == "weighted" else None)
    mode = "derive" if topo == "unit-derive" else "auto"
    ls, csr, eng = engine_for(st)
    try:
        full = Sweep(eng, mode=mode)
        full.run()
        want = sweep_digests(full)
        full.close()
    finally:
        eng.close()
    m = Multi([0, 0])
    try:
        m.load(csr)
        ms = MultiSweep(m, mode=mode)
        ms.run()
        got = ms.digests()
        for r in range(m.V):
            assert np.array_equal(got[r], want[r]), r
        a, b = ms.part_roots(0), ms.part_roots(1)
        assert np.intersect1d(a, b).size == 0 and a.size + b.size == m.V
        assert ms.owner(int(a[0])) == 0 and ms.owner(int(b[0])) == 1
        ms.close()
    finally:
        m.close()


def test_linkstate_all_sources_uses_the_sweep():
    st = drained_fabric(5, 4, seed=1, down=0.0)
    p = LinkState(stream=st)
    names = p.node_names()
    runs0 = p.spf_runs
    d_all = p.all_sources_digests()
    st_ = p.sweep_stats()
    assert st_["sweeps"] == 1 and st_["mode"] in ("lds", "derive")
    assert p.spf_runs - runs0 == len(names)
    q = LinkState(stream=st)
    d_batch = q.digests(names)
    assert np.array_equal(d_all, d_batch)
    # getSpfResult of any node now comes from the sweep's rows, no new runs
    o = Oracle(st)
    runs1 = p.spf_runs
    for r in names[:: max(1, len(names) // 12)]:
        assert p.spf_text(r) == o.spf_text(r), r
    assert p.spf_runs == runs1
    assert p.sweep_stats()["rows_copied"] > 0


def test_linkstate_multi_device_prefetch_and_route_dbs():
    """odl_create_multi over two slots of device 0: an all-nodes route build
    takes the sweep (parts per slot) and equals the single-device build."""
    st = T.fabric(pods=4, planes=4)
    a = LinkState(stream=st, devices=[0, 0])
    b = LinkState(stream=st)
    names = a.node_names()
    prefixes = {f"10.{i // 256}.{i % 256}.0/24": [(n, "ip", "ecmp", 0, None)]
                for i, n in enumerate(names[::3])}
    ra = a.route_dbs(names, prefixes)
    sa = a.sweep_stats()
    assert sa["sweeps"] == 1 and sa["devices"] == 2
    rb = b.route_dbs(names, prefixes)
    assert ra == rb
    assert np.array_equal(a.all_sources_digests(), b.digests(names))


def test_sweep_invalidated_by_graph_change():
    st = T.fabric(pods=3, planes=2)
    ls, csr, eng = engine_for(st)
    try:
        sw = Sweep(eng)
        sw.run()
        eng.update_links([(0, 0, int(csr["metric"][0]), int(csr["metric"][0]))], version=2)
        with pytest.raises(EngineError):
            sw.run()
        sw.close()
    finally:
        eng.close()


def test_leaf_derive_rejects_a_non_uniform_group():
    """ospf_leaf_derive_dev checks that a group's roots share their slot table
    (error bit 128 at ospf_sync) instead of deriving wrong rows."""
    import torch
    st = drained_fabric(4, 4, seed=5, drain=0.0, down=0.0)
    ls, csr, eng = engine_for(st)
    try:
        names = ls.node_names()
        V = eng.V
        racks = [i for i, n in enumerate(names) if n.startswith("3-")]
        a = racks[0]
        pod_a = names[a].split("-")[1]
        b = next(r for r in racks if names[r].split("-")[1] != pod_a)
        dev = torch.device("cuda", 0)
        pitch = eng.lev_pitch
        allv = np.arange(V, dtype=np.uint32)
        lev = torch.empty((V, pitch), dtype=torch.uint8, device=dev)
        d_all = torch.from_numpy(allv.view(np.int32)).to(dev)
        eng.levels_dev(d_all.data_ptr(), V, lev.data_ptr())
        roots = torch.from_numpy(np.array([a, b], np.uint32).view(np.int32)).to(dev)
        grp = torch.from_numpy(np.array([0, 2], np.uint32).view(np.int32)).to(dev)
        nh = torch.empty((2, V), dtype=torch.int32, device=dev)
        rc = eng._L.ospf_leaf_derive_dev(eng._h, roots.data_ptr(), 2, grp.data_ptr(), 1, 8,
                                         lev.data_ptr(), pitch, d_all.data_ptr(), None,
                                         nh.data_ptr(), None, None)
        assert rc == 0
        with pytest.raises(EngineError):
            eng.sync()
    finally:
        eng.close()


@pytest.mark.parametrize("seed", range(3))
def test_twin_derive_forced_on_random_and_drained_graphs(seed, monkeypatch):
    """spf_twin.hip on every <= 4-word class (OSPF_SWEEP_TWIN=1 skips the
    benefit test): random unit graphs (few twins: classes of one, the patch
    path at every neighbour), a drained fabric (racks with a down link leave
    their pod's class) and a grid with overloaded nodes -- all equal to the
    batch path bit for bit."""
    monkeypatch.setenv("OSPF_SWEEP_TWIN", "1")
    stream, _ = random_stream(seed + 20, n=60, unit=True)
    _, _, eng = engine_for(stream)
    try:
        check_sweep_vs_batch(eng, "derive")
        check_sweep_vs_batch(eng, "derive", hop=True)
    finally:
        eng.close()
    _, _, eng = engine_for(drained_fabric(5, 4, seed=seed, drain=0.08, down=0.05))
    try:
        check_sweep_vs_batch(eng, "derive")
    finally:
        eng.close()
    dbs = T.grid(14).to_dbs()
    for d in dbs[seed::17]:
        d.overloaded = True
    from openr_amd.adjdb import AdjDbStream
    _, _, eng = engine_for(AdjDbStream.from_dbs(dbs))
    try:
        check_sweep_vs_batch(eng, "derive")
    finally:
        eng.close()


def test_lds_sweep_grid31_every_root_vs_oracle():
    """BASELINE config 2 (all-sources SPF + ECMP next hops on the ~1,000-node
    grid, LDS-resident per-root work): the 31 x 31 grid's sweep takes the LDS
    path in one launch; every one of the 961 roots' digests equals the
    CSR-Dijkstra restatement, rows equal the batch path for a sample, and
    the other sweep paths agree."""
    st = T.grid(31)
    ls, csr, eng = engine_for(st)
    try:
        sw = Sweep(eng)
        assert sw.mode == "lds" and sw.n_launches == 1
        sw.run()
        eng.sync()
        got = sweep_digests(sw)
        names = ls.node_names()
        want = Oracle(st).fast_digests(names)
        bad = [names[r] for r in range(eng.V) if not np.array_equal(got[r], want[r])]
        assert not bad, bad[:8]
        sw.close()
        check_sweep_vs_batch(eng, "lds", rows_for=np.arange(0, eng.V, 13))
        check_sweep_vs_batch(eng, "derive", rows_for=np.arange(0, eng.V, 29))
    finally:
        eng.close()


@pytest.mark.parametrize("seed", range(3))
def test_lds_sweep_wide_rows_and_drains(seed):
    """Spines with 40 distinct neighbours (2 next-hop words), drained switches
    (overloaded nodes never relay) and down links: the LDS sweep == the batch
    path bit for bit, dist and next-hop rows included, and == the CPU
    restatement's digests."""
    st = drained_fabric(40, 2, seed=seed, drain=0.06, down=0.04)
    ls, csr, eng = engine_for(st)
    try:
        if not eng._L.ospf_lds_sweep_fits(eng._h, 0, 2):
            pytest.skip("graph does not fit this device's LDS")
        check_sweep_vs_batch(eng, "lds", rows_for=np.arange(0, eng.V, 5), want_mode="lds")
        check_sweep_vs_batch(eng, "lds", hop=True, rows_for=np.arange(0, eng.V, 17))
        names = ls.node_names()
        want = Oracle(st).fast_digests(names)
        sw = Sweep(eng, mode="lds")
        sw.run()
        got = sweep_digests(sw)
        assert all(np.array_equal(got[r], want[r]) for r in range(eng.V))
        sw.close()
    finally:
        eng.close()


def test_lds_sweep_direct_abi_and_limits():
    """ospf_lds_sweep_dev straight through the C ABI: a path graph deeper than
    255 levels (u16 levels), a repeated root, nh_words wider than needed
    (upper words zero), and OSPF_E_RANGE for a graph past the LDS budget."""
    import torch
    from openr_amd.adjdb import AdjDbStream
    from graphs import path_dbs
    st = AdjDbStream.from_dbs(path_dbs(600))
    ls, csr, eng = engine_for(st)
    try:
        V = eng.V
        dev = torch.device("cuda", 0)
        roots = np.array([0, V - 1, 0, 299], np.uint32)
        d_roots = torch.from_numpy(roots.view(np.int32)).to(dev)
        dist = torch.empty((4, V), dtype=torch.int32, device=dev)
        nh = torch.full((4, V, 2), -1, dtype=torch.int32, device=dev)
        dg = torch.zeros((4, 3), dtype=torch.int64, device=dev)
        rc = eng._L.ospf_lds_sweep_dev(eng._h, d_roots.data_ptr(), 4, 0, 2, dist.data_ptr(),
                                       nh.data_ptr(), dg.data_ptr(), None)
        assert rc == 0
        eng.sync()
        ref = eng.run(roots, 2, want_digest=True)
        assert np.array_equal(dist.cpu().numpy().view(np.uint32), ref["dist"])
        assert np.array_equal(nh.cpu().numpy().view(np.uint32), ref["nh"])
        assert np.array_equal(dg.cpu().numpy().view(np.uint64), ref["digest"])
        assert ref["dist"][1].max() == V - 1  # 599 levels deep
    finally:
        eng.close()
    big = T.grid(100)
    _, _, eng = engine_for(big)
    try:
        assert not eng._L.ospf_lds_sweep_fits(eng._h, 0, 1)
        with pytest.raises(EngineError):
            Sweep(eng, mode="lds")
    finally:
        eng.close()


@pytest.mark.parametrize("seed", range(3))
def test_twin_levels_forced_and_off(seed, monkeypatch):
    """ospf_twin_levels_dev inside the derive sweep (fabric switches' rows
    from a rack row of their pod and a spine row of their plane): forced on
    (OSPF_SWEEP_TWINLV=1) for drained fabrics and random graphs, and turned
    off (OSPF_SWEEP_NOTWINLV=1): both == the batch path bit for bit, and ==
    the CPU restatement's digests on the fabric."""
    st = drained_fabric(7, 4, seed=seed + 3, drain=0.07, down=0.05)
    # pipeline stages: one stage, or as many as the derived groups allow
    monkeypatch.setenv("OSPF_SWEEP_STAGES", "1" if seed == 0 else "8")
    for env in ("OSPF_SWEEP_TWINLV", "OSPF_SWEEP_NOTWINLV"):
        monkeypatch.setenv(env, "1")
        ls, csr, eng = engine_for(st)
        try:
            check_sweep_vs_batch(eng, "derive", rows_for=np.arange(0, eng.V, 3))
            names = ls.node_names()
            want = Oracle(st).fast_digests(names)
            sw = Sweep(eng, mode="derive")
            sw.run()
            got = sweep_digests(sw)
            assert all(np.array_equal(got[r], want[r]) for r in range(eng.V)), env
            if env == "OSPF_SWEEP_TWINLV":
                assert any(p["name"].startswith("twin_levels") for p in sw.profile(1))
            sw.close()
        finally:
            eng.close()
        monkeypatch.delenv(env)
    monkeypatch.setenv("OSPF_SWEEP_TWINLV", "1")
    stream, _ = random_stream(seed + 40, n=80, unit=True, p=0.1)
    _, _, eng = engine_for(stream)
    try:
        check_sweep_vs_batch(eng, "derive")
        check_sweep_vs_batch(eng, "derive", hop=True)
    finally:
        eng.close()
