#!/usr/bin/env python3
"""Transcribe the reference's own known-answer tests for the SPF path into
JSON fixtures (tests/golden/*.json).

Every expectation below is copied by hand from the cited reference test
(dgrnbrg-meta/openr @ 2025-02-28, openr/decision/tests/...); none is computed by
the oracle. The only computed thing is the *ingest order* of
``getLinkState(adjMap)`` (DecisionTestUtils.cpp:15-45), which iterates a
``std::unordered_map<int, ...>``: that order is libstdc++ behaviour, obtained
from ``oracle.intmap_order`` (which builds the same map type).

Route-level expectations (DecisionTest.cpp) are stored as next-hop sets of
``[ifName, metric, push_labels]`` for node-loopback prefixes; tests/golden_eval.py
rebuilds them from LinkState results exactly as SpfSolver does
(getNextHopsWithMetric/getNextHopsThrift SpfSolver.cpp:1043-1285 for SP_ECMP,
selectBestPathsKsp2 SpfSolver.cpp:847-973 for KSP2_ED_ECMP).

Run:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.abspath(os.path.join(HERE, "..", "..")))

from oracle import intmap_order  # noqa: E402  (libstdc++ unordered_map order only)


def adj(other, ifn, oif, metric=1, label=0, overloaded=False, weight=1):
    return dict(other=str(other), if_name=ifn, other_if=oif, metric=metric, label=label,
                overloaded=overloaded, weight=weight)


def db(name, adjs, label=0, overloaded=False, delete=False):
    return dict(name=str(name), adjs=adjs, node_label=label, overloaded=overloaded,
                delete=delete)


def adjmap_dbs(adjmap):
    """getLinkState(adjMap) (DecisionTestUtils.cpp:15-45)."""
    order = intmap_order([k for k, _ in adjmap])
    m = dict(adjmap)
    out = []
    for node in order:
        par = {}
        adjs = []
        for item in m[node]:
            other, metric = (item, 1) if isinstance(item, int) else item
            k = par.get(other, 0)
            par[other] = k + 1
            adjs.append(adj(other, f"{node}/{other}/{k}", f"{other}/{node}/{k}", metric,
                            (node << 16) + other))
        out.append(db(node, adjs, node))
    return out


fixtures = []

# ---------------------------------------------------------------------------
# LinkStateTest.BasicOperation — openr/decision/tests/LinkStateTest.cpp:139-209
n1, n2, n3 = "node1", "node2", "node3"
a12 = adj(n2, "if2", "if1", 1, 1)
a13 = adj(n3, "if3", "if1", 1, 1)
a21 = adj(n1, "if1", "if2", 1, 1)
a23 = adj(n3, "if3", "if2", 1, 1)
a31 = adj(n1, "if1", "if3", 1, 1)
a32 = adj(n2, "if2", "if3", 1, 1)
L1, L2, L3 = "node1%if2|node2%if1", "node2%if3|node3%if2", "node1%if3|node3%if1"
fixtures.append(dict(
    name="linkstate_basic_operation",
    source="openr/decision/tests/LinkStateTest.cpp:139-209",
    steps=[
        dict(dbs=[db(n1, [a12, a13], 1)], expect_changes=[[False, None, None, None]]),
        dict(dbs=[db(n2, [a21, a23], 2)], expect_changes=[[True, None, None, 1]]),
        dict(dbs=[db(n3, [a31, a32], 3)], expect_changes=[[True, None, None, 2]],
             checks=[dict(kind="links", node=n1, expect=[L1, L3]),
                     dict(kind="links", node=n2, expect=[L1, L2]),
                     dict(kind="links", node=n3, expect=[L2, L3]),
                     dict(kind="links", node="node4", expect=[]),
                     dict(kind="overloaded", node=n1, expect=False)]),
        dict(dbs=[db(n1, [a12, a13], 1, overloaded=True)],
             expect_changes=[[True, None, None, None]],
             checks=[dict(kind="overloaded", node=n1, expect=True)]),
        dict(dbs=[db(n1, [a12, a13], 1, overloaded=True)],
             expect_changes=[[False, None, None, None]]),
        dict(dbs=[db(n1, [a12, a13], 1, overloaded=False)],
             expect_changes=[[True, None, None, None]],
             checks=[dict(kind="overloaded", node=n1, expect=False)]),
        dict(dbs=[db(n1, [a13], 1)], expect_changes=[[True, None, None, None]],
             checks=[dict(kind="links", node=n1, expect=[L3]),
                     dict(kind="links", node=n2, expect=[L2]),
                     dict(kind="links", node=n3, expect=[L2, L3])]),
        dict(dbs=[db(n1, [], 0, delete=True)], expect_changes=[[True, None, None, None]],
             checks=[dict(kind="links", node=n1, expect=[]),
                     dict(kind="links", node=n2, expect=[L2]),
                     dict(kind="links", node=n3, expect=[L2])]),
    ]))

# ---------------------------------------------------------------------------
# LinkStateTest.UcmpTest — openr/decision/tests/LinkStateTest.cpp:330-483
# (kDefaultAdjWeight = 1, openr/common/Constants.h:238; adjacency weights
# default to it, LsdbUtil.h:143-152)
_ucmp_tree = [(1, [2, 3]), (2, [1, 4, 5, 6]), (3, [1, 6]), (4, [2]), (5, [2]), (6, [2, 3])]
fixtures.append(dict(
    name="linkstate_ucmp",
    source="openr/decision/tests/LinkStateTest.cpp:330-483",
    steps=[
        dict(dbs=adjmap_dbs(_ucmp_tree), checks=[
            # LWP (SP_UCMP_ADJ_WEIGHT_PROPAGATION), :341-383
            dict(kind="ucmp", root="1", leaves={"4": 2, "5": 1, "6": 1}, algo="adj",
                 expect_size=6, expect={
                     "2": {"weight": 3, "hops": {"2/4/0": 2, "2/5/0": 1, "2/6/0": 1}},
                     "3": {"weight": 1, "hops": {"3/6/0": 1}},
                     "1": {"weight": 2, "hops": {"1/2/0": 3, "1/3/0": 1}}}),
            # AWP (SP_UCMP_PREFIX_WEIGHT_PROPAGATION), :395-438
            dict(kind="ucmp", root="1", leaves={"4": 2, "5": 1, "6": 1}, algo="prefix",
                 expect_size=6, expect={
                     "2": {"weight": 4, "hops": {"2/4/0": 2, "2/5/0": 1, "2/6/0": 1}},
                     "3": {"weight": 1, "hops": {"3/6/0": 1}},
                     "1": {"weight": 5, "hops": {"1/2/0": 4, "1/3/0": 1}}}),
        ]),
    ]))
fixtures.append(dict(
    name="linkstate_ucmp_parallel_cost",
    source="openr/decision/tests/LinkStateTest.cpp:440-482",
    steps=[
        dict(dbs=adjmap_dbs([(1, [(2, 1), (5, 2), (5, 2)]), (2, [(1, 1), (3, 1), (4, 1)]),
                             (3, [(2, 1)]), (4, [(2, 1)]), (5, [(1, 2), (1, 2)])]),
             checks=[
                 dict(kind="ucmp", root="1", leaves={"3": 4, "4": 2, "5": 1}, algo="prefix",
                      expect={
                          "2": {"weight": 6, "hops": {"2/3/0": 2, "2/4/0": 1}},
                          "1": {"weight": 8,
                                "hops": {"1/2/0": 6, "1/5/0": 1, "1/5/1": 1}}}),
             ]),
    ]))

# ---------------------------------------------------------------------------
# LinkStateTest.getKthPaths — LinkStateTest.cpp:256-328
fixtures.append(dict(
    name="linkstate_kth_paths_box",
    source="openr/decision/tests/LinkStateTest.cpp:256-290",
    steps=[dict(
        dbs=adjmap_dbs([(1, [(2, 10), (3, 5)]), (2, [(1, 10), (4, 15), (4, 35)]),
                        (3, [(1, 5), (4, 20)]), (4, [(2, 15), (3, 20), (2, 35)])]),
        checks=[
            dict(kind="kth_paths", src="2", dst="4", k=1, expect_sizes=[1],
                 expect_first_link_metric_from_src=15),
            dict(kind="kth_paths", src="2", dst="4", k=2, expect_sizes_unordered=[3, 1],
                 expect_path_cost=35),
        ])]))
fixtures.append(dict(
    name="linkstate_kth_paths_full_mesh_parallel",
    source="openr/decision/tests/LinkStateTest.cpp:292-327",
    steps=[dict(
        dbs=adjmap_dbs([(1, [2, 2, 3, 3, 4, 4]), (2, [1, 1, 3, 3, 4, 4]),
                        (3, [1, 1, 2, 2, 4, 4]), (4, [1, 1, 2, 2, 3, 3])]),
        checks=[
            dict(kind="kth_paths", src="2", dst="4", k=1, expect_sizes=[1, 1]),
            dict(kind="kth_paths", src="2", dst="4", k=2, expect_sizes=[2, 2, 2, 2]),
            dict(kind="kth_paths_edge_disjoint", src="2", dst="4", ks=[1, 2]),
        ])]))

# ---------------------------------------------------------------------------
# DecisionTest constants — openr/decision/tests/DecisionTest.cpp:46-106
def dadj(me, other, metric=10, overloaded=False):
    return adj(other, f"{me}/{other}", f"{other}/{me}", metric, 100000 + other,
               overloaded=overloaded)


def nh(me, other, metric, labels=()):
    return [f"{me}/{other}", metric, list(labels)]


# SimpleRingTopologyFixture (DecisionTest.cpp:1902-2025): 1-2, 1-3, 2-4, 3-4
ring = [db(1, [dadj(1, 2), dadj(1, 3)], 1), db(2, [dadj(2, 1), dadj(2, 4)], 2),
        db(3, [dadj(3, 1), dadj(3, 4)], 3), db(4, [dadj(4, 2), dadj(4, 3)], 4)]
ring_changes = [[False, False, True, None], [True, False, True, None],
                [True, False, True, None], [True, False, True, None]]
fixtures.append(dict(
    name="decision_simple_ring_shortest_path",
    source="openr/decision/tests/DecisionTest.cpp:2027-2135",
    steps=[dict(dbs=ring, expect_changes=ring_changes, checks=[
        dict(kind="ecmp_all", nodes=["1", "2", "3", "4"]),
        dict(kind="spf_runs", expect=4),
        dict(kind="ecmp", src="1", dst="4", expect=[nh(1, 2, 20), nh(1, 3, 20)]),
        dict(kind="ecmp", src="1", dst="3", expect=[nh(1, 3, 10)]),
        dict(kind="ecmp", src="1", dst="2", expect=[nh(1, 2, 10)]),
        dict(kind="ecmp", src="2", dst="4", expect=[nh(2, 4, 10)]),
        dict(kind="ecmp", src="2", dst="3", expect=[nh(2, 1, 20), nh(2, 4, 20)]),
        dict(kind="ecmp", src="2", dst="1", expect=[nh(2, 1, 10)]),
        dict(kind="ecmp", src="3", dst="4", expect=[nh(3, 4, 10)]),
        dict(kind="ecmp", src="3", dst="2", expect=[nh(3, 1, 20), nh(3, 4, 20)]),
        dict(kind="ecmp", src="3", dst="1", expect=[nh(3, 1, 10)]),
        dict(kind="ecmp", src="4", dst="3", expect=[nh(4, 3, 10)]),
        dict(kind="ecmp", src="4", dst="2", expect=[nh(4, 2, 10)]),
        dict(kind="ecmp", src="4", dst="1", expect=[nh(4, 2, 20), nh(4, 3, 20)]),
    ])]))

fixtures.append(dict(
    name="decision_simple_ring_ksp2",
    source="openr/decision/tests/DecisionTest.cpp:2541-2712",
    steps=[
        dict(dbs=ring, expect_changes=ring_changes, checks=[
            dict(kind="ksp2_all", nodes=["1", "2", "3", "4"]),
            dict(kind="spf_runs", expect=16),
            dict(kind="ksp2", src="1", dst="4", expect=[nh(1, 2, 20, [4]), nh(1, 3, 20, [4])]),
            dict(kind="ksp2", src="1", dst="3", expect=[nh(1, 3, 10), nh(1, 2, 30, [3, 4])]),
            dict(kind="ksp2", src="1", dst="2", expect=[nh(1, 2, 10), nh(1, 3, 30, [2, 4])]),
            dict(kind="ksp2", src="2", dst="4", expect=[nh(2, 4, 10), nh(2, 1, 30, [4, 3])]),
            dict(kind="ksp2", src="2", dst="3", expect=[nh(2, 1, 20, [3]), nh(2, 4, 20, [3])]),
            dict(kind="ksp2", src="2", dst="1", expect=[nh(2, 1, 10), nh(2, 4, 30, [1, 3])]),
            dict(kind="ksp2", src="3", dst="4", expect=[nh(3, 4, 10), nh(3, 1, 30, [4, 2])]),
            dict(kind="ksp2", src="3", dst="2", expect=[nh(3, 1, 20, [2]), nh(3, 4, 20, [2])]),
            dict(kind="ksp2", src="3", dst="1", expect=[nh(3, 1, 10), nh(3, 4, 30, [1, 2])]),
            dict(kind="ksp2", src="4", dst="3", expect=[nh(4, 3, 10), nh(4, 2, 30, [3, 1])]),
            dict(kind="ksp2", src="4", dst="2", expect=[nh(4, 2, 10), nh(4, 3, 30, [2, 1])]),
            dict(kind="ksp2", src="4", dst="1", expect=[nh(4, 2, 20, [1]), nh(4, 3, 20, [1])]),
        ]),
        # adjacencyDb1.adjacencies[0] (1->2) overloaded, node 3 overloaded
        dict(dbs=[db(1, [dadj(1, 2, overloaded=True), dadj(1, 3)], 1),
                  db(3, [dadj(3, 1), dadj(3, 4)], 3, overloaded=True)],
             expect_changes=[[True, None, None, None], [True, None, None, None]],
             checks=[
                 dict(kind="ksp2", src="1", dst="4", expect=None),
                 dict(kind="ksp2", src="1", dst="3", expect=[nh(1, 3, 10)]),
                 dict(kind="ksp2", src="1", dst="2", expect=None),
             ]),
    ]))

# SimpleRingMeshTopologyFixture (DecisionTest.cpp:1690-1813): full mesh of 4
mesh4 = [db(1, [dadj(1, 2), dadj(1, 3), dadj(1, 4)], 1),
         db(2, [dadj(2, 1), dadj(2, 3), dadj(2, 4)], 2),
         db(3, [dadj(3, 1), dadj(3, 2), dadj(3, 4)], 3),
         db(4, [dadj(4, 1), dadj(4, 2), dadj(4, 3)], 4)]
fixtures.append(dict(
    name="decision_ring_mesh_ksp2",
    source="openr/decision/tests/DecisionTest.cpp:1815-1890",
    steps=[
        dict(dbs=mesh4, expect_changes=ring_changes, checks=[
            dict(kind="ksp2", src="1", dst="4",
                 expect=[nh(1, 4, 10), nh(1, 2, 20, [4]), nh(1, 3, 20, [4])]),
            dict(kind="ksp2", src="1", dst="3",
                 expect=[nh(1, 3, 10), nh(1, 2, 20, [3]), nh(1, 4, 20, [3])]),
            dict(kind="ksp2", src="1", dst="2",
                 expect=[nh(1, 2, 10), nh(1, 3, 20, [2]), nh(1, 4, 20, [2])]),
        ]),
        dict(dbs=[db(3, [dadj(3, 1), dadj(3, 2), dadj(3, 4)], 3, overloaded=True)],
             expect_changes=[[True, None, None, None]],
             checks=[dict(kind="ksp2", src="1", dst="4",
                          expect=[nh(1, 4, 10), nh(1, 2, 20, [4])])]),
    ]))


# ParallelAdjRingTopologyFixture (DecisionTest.cpp:3445-3571)
def padj(other, ifn, oif, metric, label, overloaded=False):
    return adj(other, ifn, oif, metric, label, overloaded=overloaded)


def pring(ov12_2=False, ov34_2=False):
    return [
        db(1, [padj("2", "2/1", "1/1", 11, 201), padj("2", "2/2", "1/2", 11, 202, ov12_2),
               padj("2", "2/3", "1/3", 20, 203), padj("3", "3/1", "1/1", 11, 301)], 1),
        db(2, [padj("1", "1/1", "2/1", 11, 101), padj("1", "1/2", "2/2", 11, 102),
               padj("1", "1/3", "2/3", 20, 103), padj("4", "4/1", "2/1", 11, 401)], 2),
        db(3, [padj("1", "1/1", "3/1", 11, 101), padj("4", "4/1", "3/1", 11, 401),
               padj("4", "4/2", "3/2", 20, 402, ov34_2), padj("4", "4/3", "3/3", 20, 403)], 3),
        db(4, [padj("2", "2/1", "4/1", 11, 201), padj("3", "3/1", "4/1", 11, 301),
               padj("3", "3/2", "4/2", 20, 302), padj("3", "3/3", "4/3", 20, 303)], 4),
    ]


def pn(ifn, metric, labels=()):
    return [ifn, metric, list(labels)]


pr = pring()
pr_ov = pring(True, True)
fixtures.append(dict(
    name="decision_parallel_adj_ring_ksp2",
    source="openr/decision/tests/DecisionTest.cpp:3862-4053",
    steps=[
        dict(dbs=pr, expect_changes=[[False, None, None, None], [True, None, None, None],
                                     [True, None, None, None], [True, None, None, None]],
             checks=[
                 dict(kind="ksp2", src="1", dst="2",
                      expect=[pn("2/1", 11), pn("2/2", 11), pn("2/3", 20)]),
                 # "kspf will choose adj12_2, adj13_1" (DecisionTest.cpp:3916-3932):
                 # the only reference expectation that depends on the
                 # iteration order of parallel links (folly hash of Link).
                 dict(kind="ksp2", src="1", dst="4",
                      expect=[pn("2/2", 22, [4]), pn("3/1", 22, [4])]),
             ]),
        dict(dbs=[pr_ov[0], pr_ov[2]],
             expect_changes=[[True, None, None, None], [True, None, None, None]],
             checks=[
                 dict(kind="ksp2", src="1", dst="4", expect=[pn("2/1", 22, [4]), pn("3/1", 22, [4])]),
                 dict(kind="ksp2", src="1", dst="3", expect=[pn("3/1", 11), pn("2/1", 33, [3, 4])]),
                 dict(kind="ksp2", src="1", dst="2", expect=[pn("2/1", 11), pn("2/3", 20)]),
                 dict(kind="ksp2", src="2", dst="4", expect=[pn("4/1", 11), pn("1/1", 33, [4, 3])]),
                 dict(kind="ksp2", src="2", dst="3", expect=[pn("1/1", 22, [3]), pn("4/1", 22, [3])]),
                 dict(kind="ksp2", src="2", dst="1", expect=[pn("1/1", 11), pn("1/3", 20)]),
                 dict(kind="ksp2", src="3", dst="4", expect=[pn("4/1", 11), pn("4/3", 20)]),
                 dict(kind="ksp2", src="3", dst="2", expect=[pn("1/1", 22, [2]), pn("4/1", 22, [2])]),
                 dict(kind="ksp2", src="3", dst="1", expect=[pn("1/1", 11), pn("4/1", 33, [1, 2])]),
                 dict(kind="ksp2", src="4", dst="3", expect=[pn("3/1", 11), pn("3/3", 20)]),
                 dict(kind="ksp2", src="4", dst="2", expect=[pn("2/1", 11), pn("3/1", 33, [2, 1])]),
                 dict(kind="ksp2", src="4", dst="1", expect=[pn("2/1", 22, [1]), pn("3/1", 22, [1])]),
             ]),
    ]))

# ConnectivityTest.OverloadNodeTest (DecisionTest.cpp:1455-1553): 1-2-3, 2 overloaded
fixtures.append(dict(
    name="decision_overload_node",
    source="openr/decision/tests/DecisionTest.cpp:1455-1553",
    steps=[dict(
        dbs=[db(1, [dadj(1, 2)], 1), db(2, [dadj(2, 1), dadj(2, 3)], 2, overloaded=True),
             db(3, [dadj(3, 2)], 3)],
        expect_changes=[[False, None, None, None], [True, None, None, None],
                        [True, None, None, None]],
        checks=[
            dict(kind="ecmp", src="1", dst="2", expect=[nh(1, 2, 10)]),
            dict(kind="ecmp", src="1", dst="3", expect=None),
            dict(kind="ecmp", src="2", dst="3", expect=[nh(2, 3, 10)]),
            dict(kind="ecmp", src="2", dst="1", expect=[nh(2, 1, 10)]),
            dict(kind="ecmp", src="3", dst="2", expect=[nh(3, 2, 10)]),
            dict(kind="ecmp", src="3", dst="1", expect=None),
        ])]))

# ConnectivityTest.GraphConnectedOrPartitioned (DecisionTest.cpp:1388-1449)
for partitioned in (False, True):
    dbs = [db(1, [] if partitioned else [dadj(1, 2)], 1),
           db(2, [dadj(2, 1), dadj(2, 3)], 2),
           db(3, [] if partitioned else [dadj(3, 2)], 3)]
    fixtures.append(dict(
        name=f"decision_connectivity_{'partitioned' if partitioned else 'connected'}",
        source="openr/decision/tests/DecisionTest.cpp:1388-1449",
        steps=[dict(dbs=dbs,
                    expect_changes=[[False, False, True, None],
                                    [not partitioned, False, True, None],
                                    [not partitioned, False, True, None]],
                    checks=[dict(kind="reachable", src="1", dst="3", expect=not partitioned)])]))


# GridTopologyFixture (DecisionTest.cpp:4552-4713): n = 2..16 step 2,
# every route metric == Manhattan distance, n^2(n^2-1) unicast routes.
def grid_dbs(n):
    out = []
    for i in range(n):
        for j in range(n):
            adjs = []
            for (ii, jj, ifn, oif) in ((i, j + 1, "0/1", "0/3"), (i - 1, j, "0/2", "0/4"),
                                       (i, j - 1, "0/3", "0/1"), (i + 1, j, "0/4", "0/2")):
                if 0 <= ii < n and 0 <= jj < n:
                    nb = ii * n + jj
                    adjs.append(adj(nb, ifn, oif, 1, 100001 + nb))
            out.append(db(i * n + j, adjs, i * n + j + 1))
    return out


for n in range(2, 17, 2):
    fixtures.append(dict(
        name=f"decision_grid_{n}",
        source="openr/decision/tests/DecisionTest.cpp:4552-4713",
        steps=[dict(dbs=grid_dbs(n), checks=[dict(kind="grid_manhattan", n=n)])]))


def main():
    for fx in fixtures:
        with open(os.path.join(HERE, fx["name"] + ".json"), "w") as f:
            json.dump(fx, f, indent=1, sort_keys=True)
    print(f"wrote {len(fixtures)} fixtures")


if __name__ == "__main__":
    main()
