"""Link-event sequences ([LINK UP] / [LINK DOWN] between known nodes, metric
/ overload changes) shared by the GPU parity tests (tests/test_gpu_link_events.py:
odl::LinkState on the engine, patched in place) and the CPU tests
(tests/test_host_link_events.py: the same LinkState with every SPF on the host,
odl_set_host_spf -- GPU-free, so sanitizer builds of libopenr_decision.so and
liboracle.so can run them). Reference: LinkState::updateAdjacencyDatabase,
openr/decision/LinkState.cpp:551-756 ([LINK UP] / [LINK DOWN] :632-657, memo
clear :751-754); Decision applies one database per KvStore key
(Decision.cpp:743-765)."""
import numpy as np

from graphs import random_stream
from oracle import Oracle
from openr_amd.adjdb import AdjDb, AdjDbStream, create_adjacency
from openr_amd.linkstate import LinkState


def both(stream, host=False):
    o, p = Oracle(), LinkState()
    if host:
        p.set_host_spf(True)
    assert o.apply(stream) == p.apply(stream)
    return o, p


def apply_both(o, p, dbs):
    upd = AdjDbStream.from_dbs(dbs)
    got = p.apply(upd)
    assert o.apply(upd) == got
    return got


def withdraw(dbs_by, a, idx):
    """a's database without its idx-th adjacency (the link goes: LINK DOWN)."""
    db = dbs_by[a]
    adj = db.adjs.pop(idx)
    return db, adj


def check(o, p, names, rng, k=6, all_digests=False):
    for r in rng.choice(names, min(k, len(names)), replace=False).tolist():
        assert p.spf_text(r) == o.spf_text(r), r
        assert p.spf_text(r, False) == o.spf_text(r, False), r
    if all_digests:
        assert np.array_equal(p.digests(names), o.fast_digests(names, True, threads=8))


def link_down_up_random_graphs(seed, unit, host=False, n=40):
    """Withdraw a random adjacency (both LinkSets lose the link; parallel
    links and the ranks of the others may move), check, restore it (the link
    comes back, maybe with a new link id), check; new links between known
    nodes (two one-sided advertisements, then the link); all in place."""
    st, names = random_stream(900 + seed, n=n, p=0.15, unit=unit)
    o, p = both(st, host)
    rng = np.random.default_rng(seed)
    dbs = {d.name: d for d in st.to_dbs()}
    check(o, p, names, rng)  # (loads the engine)
    s0 = p.topology_stats()
    events = 0
    for step in range(10):
        a = names[int(rng.integers(len(names)))]
        if not dbs[a].adjs:
            continue
        i = int(rng.integers(len(dbs[a].adjs)))
        db, adj = withdraw(dbs, a, i)
        ch = apply_both(o, p, [db])
        events += 1
        check(o, p, names, rng)
        assert p.spf_runs == o.spf_runs, ("withdraw", step)
        if step % 3 == 0:  # KSP2 across the event
            s_, d_ = names[int(rng.integers(len(names)))], names[int(rng.integers(len(names)))]
            for kk in (1, 2):
                assert p.kth_paths(s_, d_, kk) == o.kth_paths(s_, d_, kk)
            assert p.spf_runs == o.spf_runs, ("ksp2", step)
        db.adjs.insert(i, adj)
        apply_both(o, p, [db])
        events += 1
        check(o, p, names, rng)
        assert p.spf_runs == o.spf_runs, ("restore", step)
        del ch
    # a brand-new link between two known nodes: a advertises first (no link
    # yet: the other side does not), then b (the link forms)
    for step in range(4):
        a, b = rng.choice(names, 2, replace=False).tolist()
        ia, ib = f"{a}-{b}-new{step}", f"{b}-{a}-new{step}"
        m1 = 1 if unit else int(rng.integers(1, 20))
        m2 = 1 if unit else int(rng.integers(1, 20))
        dbs[a].adjs.append(create_adjacency(b, ia, ib, m1))
        apply_both(o, p, [dbs[a]])
        dbs[b].adjs.append(create_adjacency(a, ib, ia, m2))
        apply_both(o, p, [dbs[b]])
        events += 1
        check(o, p, names, rng)
        assert p.spf_runs == o.spf_runs, ("new link", step)
    s1 = p.topology_stats()
    # every link event patched in place: no snapshot, no device load
    assert s1["snapshots"] == s0["snapshots"] and s1["loads"] == s0["loads"], (s0, s1)
    assert s1["link_patches"] - s0["link_patches"] == events
    assert p.spf_runs == o.spf_runs
    # all-sources sweep and every root's digest on the patched graph
    ids = p.node_names()  # all_sources_digests: node-id order
    assert np.array_equal(p.all_sources_digests(), o.fast_digests(ids, True, threads=8))
    check(o, p, names, rng, all_digests=True)


def link_events_mixed_with_metric_and_overload(host=False):
    """One database update that removes a link, adds one and changes a
    metric and an adjacency overload bit at once; then node overload."""
    st, names = random_stream(77, n=30, p=0.2)
    o, p = both(st, host)
    rng = np.random.default_rng(1)
    dbs = {d.name: d for d in st.to_dbs()}
    for step in range(8):
        a = names[int(rng.integers(len(names)))]
        db = dbs[a]
        if len(db.adjs) < 3:
            continue
        db.adjs.pop(0)
        db.adjs[0].metric = int(rng.integers(1, 50))
        db.adjs[1].overloaded = not db.adjs[1].overloaded
        c = names[int(rng.integers(len(names)))]
        if c != a:
            db.adjs.append(create_adjacency(c, f"{a}-{c}-m{step}", f"{c}-{a}-m{step}", 3))
            dbs[c].adjs.append(create_adjacency(a, f"{c}-{a}-m{step}", f"{a}-{c}-m{step}", 4))
            apply_both(o, p, [db, dbs[c]])
        else:
            apply_both(o, p, [db])
        check(o, p, names, rng)
        dbs[a].overloaded = not dbs[a].overloaded
        apply_both(o, p, [dbs[a]])
        check(o, p, names, rng)
    assert p.spf_runs == o.spf_runs


def parallel_link_ranks_after_insert(host=False):
    """Parallel links: a node whose LinkSet grows past a bucket count
    rehashes, which can reorder its links (ranks) and with them the
    pathLinks order of its neighbours' parallel groups (the engine rebuilds
    those rows too). Many links added to one hub, KSP2 and text checked."""
    n = 12
    adj = {f"n{i}": [] for i in range(n)}
    for i in range(1, n):
        for k in range(2):  # two parallel links hub - n{i}
            a, b = "n0", f"n{i}"
            adj[a].append(create_adjacency(b, f"{a}-{b}-{k}", f"{b}-{a}-{k}", 5))
            adj[b].append(create_adjacency(a, f"{b}-{a}-{k}", f"{a}-{b}-{k}", 5))
    for i in range(1, n - 1):  # a ring around the hub
        a, b = f"n{i}", f"n{i + 1}"
        adj[a].append(create_adjacency(b, f"{a}-{b}-r", f"{b}-{a}-r", 7))
        adj[b].append(create_adjacency(a, f"{b}-{a}-r", f"{a}-{b}-r", 7))
    dbs = {nm: AdjDb(nm, adj[nm], i + 1) for i, nm in enumerate(adj)}
    st = AdjDbStream.from_dbs(list(dbs.values()))
    o, p = both(st, host)
    names = sorted(dbs)
    assert p.spf_text("n1") == o.spf_text("n1")  # snapshot + engine load
    s0 = p.topology_stats()
    for step in range(30):  # hub grows: rehashes of its LinkSet
        b = f"n{1 + step % (n - 1)}"
        ia, ib = f"n0-{b}-x{step}", f"{b}-n0-x{step}"
        dbs["n0"].adjs.append(create_adjacency(b, ia, ib, 5))
        dbs[b].adjs.append(create_adjacency("n0", ib, ia, 5))
        apply_both(o, p, [dbs["n0"], dbs[b]])
        for r in names:
            assert p.spf_text(r) == o.spf_text(r), (step, r)
        for d in names[1:4]:
            assert p.kth_paths("n5", d, 2) == o.kth_paths("n5", d, 2), (step, d)
    assert p.topology_stats()["snapshots"] == s0["snapshots"]


def node_remove_add_random_graphs(seed, unit, host=False, n=40):
    """A node's database withdrawn (deleteAdjacencyDatabase: its links leave
    its peers' rows, its row leaves, ids above it move down), then restored
    (its links form again with peers that still advertise it); a brand-new
    node joining with links to known nodes; all in place on the host
    snapshot (LinkState.cpp:584-600 new node, :730-756 delete)."""
    from openr_amd.adjdb import AdjDb
    st, names = random_stream(1300 + seed, n=n, p=0.15, unit=unit)
    o, p = both(st, host)
    rng = np.random.default_rng(seed)
    dbs = {d.name: d for d in st.to_dbs()}
    check(o, p, names, rng)
    s0 = p.topology_stats()
    np0 = p.node_patches
    events = 0
    live = list(names)
    for step in range(6):
        a = live[int(rng.integers(len(live)))]
        apply_both(o, p, [AdjDb(a, delete=True)])  # the node leaves
        live.remove(a)
        events += 1
        check(o, p, live, rng)
        assert p.spf_runs == o.spf_runs, ("delete", step)
        if step % 2 == 0:  # KSP2 without it
            s_, d_ = live[int(rng.integers(len(live)))], live[int(rng.integers(len(live)))]
            for kk in (1, 2):
                assert p.kth_paths(s_, d_, kk) == o.kth_paths(s_, d_, kk)
        apply_both(o, p, [dbs[a]])  # and comes back
        live.append(a)
        events += 1
        check(o, p, live, rng)
        assert p.spf_runs == o.spf_runs, ("restore", step)
    # new nodes whose peers advertise them first (links form at once), with
    # names sorting before, between and after the others
    for step, nm in enumerate(["a-new", "r5-new", "zz-new"]):
        peers = rng.choice(live, 3, replace=False).tolist()
        mine = []
        for q in peers:
            m1 = 1 if unit else int(rng.integers(1, 20))
            m2 = 1 if unit else int(rng.integers(1, 20))
            dbs[q].adjs.append(create_adjacency(nm, f"{q}-{nm}", f"{nm}-{q}", m1))
            mine.append(create_adjacency(q, f"{nm}-{q}", f"{q}-{nm}", m2))
        apply_both(o, p, [dbs[q] for q in peers])
        dbs[nm] = AdjDb(nm, mine, 1000 + step)
        apply_both(o, p, [dbs[nm]])
        live.append(nm)
        events += 1
        check(o, p, live, rng)
        assert p.spf_runs == o.spf_runs, ("new node", step)
    s1 = p.topology_stats()
    assert s1["snapshots"] == s0["snapshots"], (s0, s1)  # no whole snapshot
    assert p.node_patches - np0 == events
    ids = p.node_names()
    assert sorted(ids) == ids and set(ids) == set(live)
    assert np.array_equal(p.all_sources_digests(), o.fast_digests(ids, True, threads=8))
    check(o, p, live, rng, all_digests=True)
    return s0, s1
