"""Route building (SpfSolver::buildRouteDb) on the
GPU SPF results: the product's C++ odl::SpfSolver against the test-side
restatement (golden_eval.RouteBuilder) evaluated over the CPU oracle, on
random graphs with multi-announcer prefixes, every forwarding type /
algorithm, prepend labels, drained announcers, label collisions and UCMP.
The restatement itself is pinned by the reference's route fixtures
(tests/golden/decision_*routes*.json, test_oracle_golden.py)."""
import dataclasses

import numpy as np
import pytest

from golden_eval import OracleLS, RouteBuilder
from openr_amd.adjdb import AdjDb, AdjDbStream, create_adjacency
from openr_amd.linkstate import LinkState

pytestmark = pytest.mark.gpu

COMBOS = [("ip", "ecmp"), ("sr_mpls", "ecmp"), ("sr_mpls", "ksp2"), ("ip", "ksp2"),
          ("ip", "ucmp_prefix"), ("ip", "ucmp_adj"), ("sr_mpls", "ucmp_prefix")]


def random_routing_case(seed, n=24, p=0.2, wmax=20):
    rng = np.random.default_rng(seed)
    names = [f"n{int(x)}" for x in rng.permutation(10 * n)[:n]]
    adjs = {nm: [] for nm in names}
    k = 0
    for i in range(n):
        for j in range(i + 1, n):
            if rng.random() > p:
                continue
            for _ in range(2 if rng.random() < 0.2 else 1):
                a, b = names[i], names[j]
                ia, ib = f"{a}-{b}-{k}", f"{b}-{a}-{k}"
                adjs[a].append(create_adjacency(
                    b, ia, ib, int(rng.integers(1, wmax + 1)), 100000 + 2 * k,
                    weight=int(rng.integers(1, 4)), overloaded=bool(rng.random() < 0.08)))
                adjs[b].append(create_adjacency(
                    a, ib, ia, int(rng.integers(1, wmax + 1)), 100001 + 2 * k,
                    weight=int(rng.integers(1, 4))))
                k += 1
    labels = [i + 1 for i in range(n)]
    labels[1] = 0                 # non-SR node: no node-label route, voids KSP2 paths
    labels[3] = labels[2]         # label collision: the smaller name keeps it
    labels[4] = 0x100000          # invalid (> 20 bits)
    dbs = [AdjDb(nm, adjs[nm], labels[i], overloaded=bool(rng.random() < 0.1))
           for i, nm in enumerate(names)]
    prefixes = {}
    for q in range(30):
        ents = []
        for node in rng.choice(names, size=int(rng.integers(1, 4)), replace=False):
            fwd, algo = COMBOS[int(rng.integers(0, len(COMBOS)))]
            w = int(rng.integers(0, 4)) * 1000
            pl = int(rng.integers(200, 300)) if rng.random() < 0.2 else None
            ents.append([str(node), fwd, algo, w, pl])
        prefixes[f"10.{seed % 200}.{q}.0/24"] = ents
    return dbs, names, prefixes


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("ucmp", [False, True])
def test_route_dbs_match_restatement(seed, ucmp):
    dbs, names, prefixes = random_routing_case(seed)
    stream = AdjDbStream.from_dbs(dbs)
    o, p = OracleLS(), LinkState()
    assert o.apply(stream) == p.apply(stream)
    cur = {d.name: dataclasses.asdict(d) for d in dbs}
    rb = RouteBuilder(o, cur, ucmp=ucmp)
    want = {me: rb.build(me, prefixes) for me in names + ["unknown"]}
    got = p.route_dbs(names + ["unknown"], prefixes, ucmp=ucmp)  # odl_route_db_bin
    # the binary records decode to exactly the text ABI's databases
    assert got == p.route_dbs(names + ["unknown"], prefixes, ucmp=ucmp, binary=False)
    assert got["unknown"] is None
    n_routes = 0
    for me in names:
        assert got[me] == want[me], me
        n_routes += len(got[me]) - 1
    assert n_routes > len(names)


def test_route_dbs_without_labels():
    dbs, names, prefixes = random_routing_case(11)
    stream = AdjDbStream.from_dbs(dbs)
    o, p = OracleLS(), LinkState()
    o.apply(stream)
    p.apply(stream)
    cur = {d.name: dataclasses.asdict(d) for d in dbs}
    rb = RouteBuilder(o, cur, node_labels=False, adj_labels=False)
    got = p.route_dbs(names, prefixes, node_labels=False, adj_labels=False)
    for me in names:
        assert got[me] == rb.build(me, prefixes)
        assert not any(k[0] == "M" for k in got[me] if k != "routes")


@pytest.mark.parametrize("seed", range(4))
def test_best_route_selection_matches_restatement(seed):
    """enableBestRouteSelection (SpfSolver.cpp:658-663; selectRoutes
    SHORTEST_DISTANCE + selectBestNodeArea, LsdbUtil.cpp:758-880) on random
    multi-announcer prefixes with random prefix metrics and origin types:
    the product's routes and best-route results equal the restatement's."""
    dbs, names, prefixes = random_routing_case(100 + seed)
    rng = np.random.default_rng(seed)
    for ents in prefixes.values():
        for e in ents:
            met = [int(rng.integers(0, 3)) * 100, int(rng.integers(0, 2)) * 50,
                   int(rng.integers(0, 3))]
            e += [None, None, met, [None, "bgp", "bgpmv"][int(rng.integers(0, 3))]]
    stream = AdjDbStream.from_dbs(dbs)
    o, p = OracleLS(), LinkState()
    assert o.apply(stream) == p.apply(stream)
    cur = {d.name: dataclasses.asdict(d) for d in dbs}
    rb = RouteBuilder(o, cur, best_route_selection=True)
    got = p.route_dbs(names, prefixes, best_route_selection=True)
    n_best = 0
    for me in names:
        assert got[me] == rb.build(me, prefixes), me
        n_best += len((got[me] or {}).get("best", {}))
    assert n_best > len(names)
