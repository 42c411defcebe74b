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


def grid_prefix(node):
    """nodeToPrefixV6 (DecisionTest.cpp:4595-4598)."""
    return f"::ffff:10.1.{node // 256}.{node % 256}/128"


for n in range(2, 17, 2):
    fixtures.append(dict(
        name=f"decision_grid_{n}",
        source="openr/decision/tests/DecisionTest.cpp:4552-4713",
        steps=[dict(dbs=grid_dbs(n), checks=[
            dict(kind="grid_manhattan", n=n),
            # ShortestPathTest (:4668-4713): 2n^4 + 3n^2 - 4n routes, corner
            # to corner metrics = Manhattan distance
            dict(kind="route_map", nodes=[str(i) for i in range(n * n)],
                 prefixes={grid_prefix(i): [[str(i), "ip", "ecmp", 0, None]]
                           for i in range(n * n)},
                 expect_size=2 * n ** 4 + 3 * n ** 2 - 4 * n,
                 expect_metric={f"0|U|{grid_prefix(n * n - 1)}": 2 * (n - 1),
                                f"{n - 1}|U|{grid_prefix(n * (n - 1))}": 2 * (n - 1)}),
        ])]))


# ---------------------------------------------------------------------------
# Route-DB fixtures: SpfSolver::buildRouteDb over the link state. A check
# "route_map" lists the nodes whose route DBs the reference's getRouteMap
# (DecisionTest.cpp:311-329) collects, the prefix entries, and the reference's
# assertions: the map size (one key per (node, prefix | label)), exact next-hop
# sets (validatePopLabelRoute / validateAdjLabelRoutes :363-386 included) and
# per-node route counts. Next hop = [ifName, neighbor, metric, mpls action,
# labels, ucmp weight] (createNextHopFromAdj :234-252; the address field is
# the adjacency's, not modelled).
def H(ifn, nbr, metric, op="", labels=(), w=0):
    return [ifn, str(nbr), metric, op, list(labels), w]


POP = ["", "", 0, "POP", [], 0]  # labelPopNextHop (DecisionTest.cpp:161-166)
ADDR = {1: "::ffff:10.1.1.1/128", 2: "::ffff:10.2.2.2/128", 3: "::ffff:10.3.3.3/128",
        4: "::ffff:10.4.4.4/128"}  # addr1..addr4 (DecisionTest.cpp:108-111)


def loopbacks(nodes):
    """prefixDb1..4 (DecisionTest.cpp:137-140): createPrefixEntry(addrN),
    forwarding IP / SP_ECMP (the thrift defaults)."""
    return {ADDR[n]: [[str(n), "ip", "ecmp", 0, None]] for n in nodes}


def route_map(nodes, prefixes, **kw):
    return dict(kind="route_map", nodes=[str(n) for n in nodes], prefixes=prefixes, **kw)


def adj_routes(node, adjs):
    """validateAdjLabelRoutes (DecisionTest.cpp:363-377)."""
    return {f"{node}|M|{a['label']}": [H(a["if_name"], a["other"], a["metric"], "PHP")]
            for a in adjs}


# ShortestPathTest.* (DecisionTest.cpp:473-609)
fixtures.append(dict(
    name="decision_route_unreachable_nodes",
    source="openr/decision/tests/DecisionTest.cpp:473-505",
    steps=[dict(dbs=[db(1, [], 0), db(2, [], 0)],
                expect_changes=[[False, None, None, None], [False, None, None, None]],
                checks=[route_map([1, 2], loopbacks([1, 2]),
                                  expect_counts={"1": [0, 0], "2": [0, 0]})])]))
fixtures.append(dict(
    name="decision_route_missing_neighbor_adjdb",
    source="openr/decision/tests/DecisionTest.cpp:512-541",
    steps=[dict(dbs=[db(1, [dadj(1, 2)], 0)], expect_changes=[[False, None, None, None]],
                checks=[route_map([1], loopbacks([1, 2]), expect_counts={"1": [0, 0]})])]))
fixtures.append(dict(
    name="decision_route_empty_neighbor_adjdb",
    source="openr/decision/tests/DecisionTest.cpp:549-586",
    steps=[dict(dbs=[db(1, [dadj(1, 2)], 0), db(2, [], 0)],
                expect_changes=[[False, None, None, None], [False, None, None, None]],
                checks=[route_map([1, 2], loopbacks([1, 2]),
                                  expect_counts={"1": [0, None], "2": [0, None]})])]))
fixtures.append(dict(
    name="decision_route_unknown_node",
    source="openr/decision/tests/DecisionTest.cpp:591-609",
    steps=[dict(dbs=[], checks=[route_map([1, 2], {}, expect_counts={"1": None, "2": None})])]))

# SpfSolver.AdjacencyUpdate (DecisionTest.cpp:614-759). The next-hop address
# updates (:664-718) change a field this path does not model and are left out.
_au12 = adj("2", "1/2", "2/1", 10, 111)
_au21 = adj("1", "2/1", "1/2", 10, 222)
fixtures.append(dict(
    name="decision_spf_solver_adjacency_update",
    source="openr/decision/tests/DecisionTest.cpp:614-759",
    steps=[
        dict(dbs=[db(1, [dadj(1, 2)], 1)], expect_changes=[[False, None, True, None]]),
        dict(dbs=[db(2, [dadj(2, 1)], 2)], expect_changes=[[True, None, True, None]],
             checks=[route_map([1, 2], loopbacks([1, 2]),
                               expect_counts={"1": [1, 3], "2": [1, 3]})]),
        dict(dbs=[db(1, [_au12], 1)], expect_changes=[[False, True, None, None]]),
        dict(dbs=[db(2, [_au21], 2)], expect_changes=[[False, True, None, None]]),
        dict(dbs=[db(1, [_au12], 11)], expect_changes=[[False, False, True, None]]),
        dict(dbs=[db(2, [_au21], 22)], expect_changes=[[False, False, True, None]]),
    ]))

# MplsRoutes.BasicTest (DecisionTest.cpp:765-812): 1 -> 2 not bidirectional,
# 2 <-> 3; node 2 has no node label
_m1 = db(1, [dadj(1, 2)], 1)
fixtures.append(dict(
    name="decision_mpls_routes_basic",
    source="openr/decision/tests/DecisionTest.cpp:765-812",
    steps=[dict(
        dbs=[_m1, _m1, db(2, [dadj(2, 3)], 0), db(3, [dadj(3, 2)], 3)],
        expect_changes=[[False, False, True, None], [False, False, False, None],
                        [False, False, False, None], [True, False, True, None]],
        checks=[route_map([1, 2, 3], {}, expect_size=5, expect={
            "1|M|1": [POP],
            "2|M|100003": [H("2/3", 3, 10, "PHP")],
            "3|M|3": [POP],
            "3|M|100002": [H("3/2", 2, 10, "PHP")]})])]))

# SimpleRingTopologyFixture.OverloadNodeTest (DecisionTest.cpp:3115-3234)
ring_pfx = loopbacks([1, 2, 3, 4])
fixtures.append(dict(
    name="decision_simple_ring_overload_node_routes",
    source="openr/decision/tests/DecisionTest.cpp:3115-3234",
    steps=[
        dict(dbs=ring, expect_changes=ring_changes),
        dict(dbs=[db(2, [dadj(2, 1), dadj(2, 4)], 2, overloaded=True),
                  db(3, [dadj(3, 1), dadj(3, 4)], 3, overloaded=True)],
             expect_changes=[[True, None, None, None], [True, None, None, None]],
             checks=[route_map([1, 2, 3, 4], ring_pfx, expect_size=32, expect={
                 f"1|U|{ADDR[3]}": [H("1/3", 3, 10)], "1|M|3": [H("1/3", 3, 10, "PHP")],
                 f"1|U|{ADDR[2]}": [H("1/2", 2, 10)], "1|M|2": [H("1/2", 2, 10, "PHP")],
                 "1|M|1": [POP], **adj_routes(1, ring[0]["adjs"]),
                 f"2|U|{ADDR[4]}": [H("2/4", 4, 10)], "2|M|4": [H("2/4", 4, 10, "PHP")],
                 f"2|U|{ADDR[3]}": [H("2/1", 1, 20), H("2/4", 4, 20)],
                 "2|M|3": [H("2/1", 1, 20, "SWAP", [3]), H("2/4", 4, 20, "SWAP", [3])],
                 f"2|U|{ADDR[1]}": [H("2/1", 1, 10)], "2|M|1": [H("2/1", 1, 10, "PHP")],
                 "2|M|2": [POP], **adj_routes(2, ring[1]["adjs"]),
                 f"3|U|{ADDR[4]}": [H("3/4", 4, 10)], "3|M|4": [H("3/4", 4, 10, "PHP")],
                 f"3|U|{ADDR[2]}": [H("3/1", 1, 20), H("3/4", 4, 20)],
                 "3|M|2": [H("3/1", 1, 20, "SWAP", [2]), H("3/4", 4, 20, "SWAP", [2])],
                 f"3|U|{ADDR[1]}": [H("3/1", 1, 10)], "3|M|1": [H("3/1", 1, 10, "PHP")],
                 "3|M|3": [POP], **adj_routes(3, ring[2]["adjs"]),
                 f"4|U|{ADDR[3]}": [H("4/3", 3, 10)], "4|M|3": [H("4/3", 3, 10, "PHP")],
                 f"4|U|{ADDR[2]}": [H("4/2", 2, 10)], "4|M|2": [H("4/2", 2, 10, "PHP")],
                 "4|M|4": [POP], **adj_routes(4, ring[3]["adjs"])})]),
    ]))

# SimpleRingTopologyFixture.OverloadLinkTest (DecisionTest.cpp:3240-3427)
_r3a = db(3, [dadj(3, 1, overloaded=True), dadj(3, 4)], 3)
_r3b = db(3, [dadj(3, 1, overloaded=True), dadj(3, 4, overloaded=True)], 3)
fixtures.append(dict(
    name="decision_simple_ring_overload_link_routes",
    source="openr/decision/tests/DecisionTest.cpp:3240-3427",
    steps=[
        dict(dbs=ring, expect_changes=ring_changes),
        dict(dbs=[_r3a], expect_changes=[[True, None, None, None]],
             checks=[route_map([1, 2, 3, 4], ring_pfx, expect_size=36, expect={
                 f"1|U|{ADDR[4]}": [H("1/2", 2, 20)], "1|M|4": [H("1/2", 2, 20, "SWAP", [4])],
                 f"1|U|{ADDR[3]}": [H("1/2", 2, 30)], "1|M|3": [H("1/2", 2, 30, "SWAP", [3])],
                 f"1|U|{ADDR[2]}": [H("1/2", 2, 10)], "1|M|2": [H("1/2", 2, 10, "PHP")],
                 "1|M|1": [POP], **adj_routes(1, ring[0]["adjs"]),
                 f"2|U|{ADDR[4]}": [H("2/4", 4, 10)], "2|M|4": [H("2/4", 4, 10, "PHP")],
                 f"2|U|{ADDR[3]}": [H("2/4", 4, 20)], "2|M|3": [H("2/4", 4, 20, "SWAP", [3])],
                 f"2|U|{ADDR[1]}": [H("2/1", 1, 10)], "2|M|1": [H("2/1", 1, 10, "PHP")],
                 "2|M|2": [POP], **adj_routes(2, ring[1]["adjs"]),
                 f"3|U|{ADDR[4]}": [H("3/4", 4, 10)], "3|M|4": [H("3/4", 4, 10, "PHP")],
                 f"3|U|{ADDR[2]}": [H("3/4", 4, 20)], "3|M|2": [H("3/4", 4, 20, "SWAP", [2])],
                 f"3|U|{ADDR[1]}": [H("3/4", 4, 30)], "3|M|1": [H("3/4", 4, 30, "SWAP", [1])],
                 "3|M|3": [POP], **adj_routes(3, _r3a["adjs"]),
                 f"4|U|{ADDR[3]}": [H("4/3", 3, 10)], "4|M|3": [H("4/3", 3, 10, "PHP")],
                 f"4|U|{ADDR[2]}": [H("4/2", 2, 10)], "4|M|2": [H("4/2", 2, 10, "PHP")],
                 f"4|U|{ADDR[1]}": [H("4/2", 2, 20)], "4|M|1": [H("4/2", 2, 20, "SWAP", [1])],
                 "4|M|4": [POP], **adj_routes(4, ring[3]["adjs"])})]),
        dict(dbs=[_r3b], expect_changes=[[True, None, None, None]],
             checks=[route_map([1, 2, 3, 4], ring_pfx, expect_size=24, expect={
                 f"1|U|{ADDR[4]}": [H("1/2", 2, 20)], "1|M|4": [H("1/2", 2, 20, "SWAP", [4])],
                 f"1|U|{ADDR[2]}": [H("1/2", 2, 10)], "1|M|2": [H("1/2", 2, 10, "PHP")],
                 "1|M|1": [POP], **adj_routes(1, ring[0]["adjs"]),
                 f"2|U|{ADDR[4]}": [H("2/4", 4, 10)], "2|M|4": [H("2/4", 4, 10, "PHP")],
                 f"2|U|{ADDR[1]}": [H("2/1", 1, 10)], "2|M|1": [H("2/1", 1, 10, "PHP")],
                 "2|M|2": [POP], **adj_routes(2, ring[1]["adjs"]),
                 "3|M|3": [POP], **adj_routes(3, _r3b["adjs"]),
                 f"4|U|{ADDR[2]}": [H("4/2", 2, 10)], "4|M|2": [H("4/2", 2, 10, "PHP")],
                 f"4|U|{ADDR[1]}": [H("4/2", 2, 20)], "4|M|1": [H("4/2", 2, 20, "SWAP", [1])],
                 "4|M|4": [POP], **adj_routes(4, ring[3]["adjs"])})]),
    ]))

# ParallelAdjRingTopologyFixture.ShortestPathTest (DecisionTest.cpp:3573-3706)
def _sw(hops, lbl):
    return [h[:3] + (["PHP", [], 0] if lbl is None else ["SWAP", [lbl], 0]) for h in hops]


_p1_4 = [H("2/2", 2, 22), H("3/1", 3, 22), H("2/1", 2, 22)]
_p2_3 = [H("1/2", 1, 22), H("1/1", 1, 22), H("4/1", 4, 22)]
_p3_2 = [H("1/1", 1, 22), H("4/1", 4, 22)]
_p4_1 = [H("2/1", 2, 22), H("3/1", 3, 22)]
fixtures.append(dict(
    name="decision_parallel_adj_ring_shortest_path_routes",
    source="openr/decision/tests/DecisionTest.cpp:3573-3706",
    steps=[dict(
        dbs=pr, expect_changes=[[False, None, None, None], [True, None, None, None],
                                [True, None, None, None], [True, None, None, None]],
        checks=[route_map([1, 2, 3, 4], ring_pfx, expect_size=44, expect={
            f"1|U|{ADDR[4]}": _p1_4, "1|M|4": _sw(_p1_4, 4),
            f"1|U|{ADDR[3]}": [H("3/1", 3, 11)], "1|M|3": [H("3/1", 3, 11, "PHP")],
            f"1|U|{ADDR[2]}": [H("2/2", 2, 11), H("2/1", 2, 11)],
            "1|M|2": _sw([H("2/2", 2, 11), H("2/1", 2, 11)], None),
            "1|M|1": [POP], **adj_routes(1, pr[0]["adjs"]),
            f"2|U|{ADDR[4]}": [H("4/1", 4, 11)], "2|M|4": [H("4/1", 4, 11, "PHP")],
            f"2|U|{ADDR[3]}": _p2_3, "2|M|3": _sw(_p2_3, 3),
            f"2|U|{ADDR[1]}": [H("1/2", 1, 11), H("1/1", 1, 11)],
            "2|M|1": _sw([H("1/2", 1, 11), H("1/1", 1, 11)], None),
            "2|M|2": [POP], **adj_routes(2, pr[1]["adjs"]),
            f"3|U|{ADDR[4]}": [H("4/1", 4, 11)], "3|M|4": [H("4/1", 4, 11, "PHP")],
            f"3|U|{ADDR[2]}": _p3_2, "3|M|2": _sw(_p3_2, 2),
            f"3|U|{ADDR[1]}": [H("1/1", 1, 11)], "3|M|1": [H("1/1", 1, 11, "PHP")],
            "3|M|3": [POP], **adj_routes(3, pr[2]["adjs"]),
            f"4|U|{ADDR[3]}": [H("3/1", 3, 11)], "4|M|3": [H("3/1", 3, 11, "PHP")],
            f"4|U|{ADDR[2]}": [H("2/1", 2, 11)], "4|M|2": [H("2/1", 2, 11, "PHP")],
            f"4|U|{ADDR[1]}": _p4_1, "4|M|1": _sw(_p4_1, 1),
            "4|M|4": [POP], **adj_routes(4, pr[3]["adjs"])})])]))

# DecisionTest.Ucmp (DecisionTest.cpp:7861-8130): UCMP on, node/adjacency
# labels off; adjacencies metric 10, adj label 0, weight 100e9
G = 10 ** 9


def uadj(me, other):
    return adj(str(other), f"{me}/{other}", f"{other}/{me}", 10, 0, weight=100 * G)


_utree = {1: [2, 3], 2: [1, 4, 5], 3: [1, 6], 4: [2], 5: [2], 6: [3]}
_udbs = [db(n, [uadj(n, o) for o in nb], n) for n, nb in _utree.items()]
_dflt = "::/0"
_uopts = dict(ucmp=True, node_labels=False, adj_labels=False)


def _ue(node, algo, w):
    return [str(node), "ip", algo, w, None]


fixtures.append(dict(
    name="decision_ucmp_routes",
    source="openr/decision/tests/DecisionTest.cpp:7861-8130",
    steps=[dict(dbs=_udbs, checks=[
        # Test 1 (:7923-8013): all SP_UCMP_PREFIX_WEIGHT_PROPAGATION
        route_map([1, 2, 3], {_dflt: [_ue(4, "ucmp_prefix", 200 * G),
                                      _ue(5, "ucmp_prefix", 100 * G),
                                      _ue(6, "ucmp_prefix", 100 * G)]}, opts=_uopts,
                  expect_counts={"1": [1, 0], "2": [1, 0], "3": [1, 0]},
                  expect_weight={f"1|{_dflt}": 400 * G, f"2|{_dflt}": 300 * G,
                                 f"3|{_dflt}": 100 * G},
                  expect={f"1|U|{_dflt}": [H("1/2", 2, 20, w=3), H("1/3", 3, 20, w=1)],
                          f"2|U|{_dflt}": [H("2/4", 4, 10, w=2), H("2/5", 5, 10, w=1)],
                          f"3|U|{_dflt}": [H("3/6", 6, 10, w=1)]}),
        # Test 2 (:8015-8071): node 6 SP_UCMP_ADJ_WEIGHT_PROPAGATION
        route_map([1, 2, 3], {_dflt: [_ue(4, "ucmp_prefix", 200 * G),
                                      _ue(5, "ucmp_prefix", 100 * G),
                                      _ue(6, "ucmp_adj", 100 * G)]}, opts=_uopts,
                  expect_counts={"1": [1, 0], "2": [1, 0], "3": [1, 0]},
                  expect_weight={f"1|{_dflt}": 200 * G, f"2|{_dflt}": 200 * G,
                                 f"3|{_dflt}": 100 * G},
                  expect={f"1|U|{_dflt}": [H("1/2", 2, 20, w=2), H("1/3", 3, 20, w=1)],
                          f"2|U|{_dflt}": [H("2/4", 4, 10, w=2), H("2/5", 5, 10, w=1)],
                          f"3|U|{_dflt}": [H("3/6", 6, 10, w=1)]}),
        # Test 3 (:8073-8129): node 6 without a weight
        route_map([1, 2, 3], {_dflt: [_ue(4, "ucmp_prefix", 200 * G),
                                      _ue(5, "ucmp_prefix", 100 * G),
                                      _ue(6, "ucmp_prefix", 0)]}, opts=_uopts,
                  expect_counts={"1": [1, 0], "2": [1, 0], "3": [1, 0]},
                  expect_weight={f"1|{_dflt}": None, f"2|{_dflt}": 300 * G,
                                 f"3|{_dflt}": None},
                  expect={f"1|U|{_dflt}": [H("1/2", 2, 20), H("1/3", 3, 20)],
                          f"2|U|{_dflt}": [H("2/4", 4, 10, w=2), H("2/5", 5, 10, w=1)],
                          f"3|U|{_dflt}": [H("3/6", 6, 10)]}),
    ])]))

# SimpleRingTopologyFixture.MultiPathTest (DecisionTest.cpp:2231-2365):
# node + adjacency labels, 12 unicast + 16 node-label + 8 adjacency routes
def _ring_full(extra=None):
    e = {
        f"1|U|{ADDR[4]}": [H("1/2", 2, 20), H("1/3", 3, 20)],
        "1|M|4": [H("1/2", 2, 20, "SWAP", [4]), H("1/3", 3, 20, "SWAP", [4])],
        f"1|U|{ADDR[3]}": [H("1/3", 3, 10)], "1|M|3": [H("1/3", 3, 10, "PHP")],
        f"1|U|{ADDR[2]}": [H("1/2", 2, 10)], "1|M|2": [H("1/2", 2, 10, "PHP")],
        "1|M|1": [POP], **adj_routes(1, ring[0]["adjs"]),
        f"2|U|{ADDR[4]}": [H("2/4", 4, 10)], "2|M|4": [H("2/4", 4, 10, "PHP")],
        f"2|U|{ADDR[3]}": [H("2/1", 1, 20), H("2/4", 4, 20)],
        "2|M|3": [H("2/1", 1, 20, "SWAP", [3]), H("2/4", 4, 20, "SWAP", [3])],
        f"2|U|{ADDR[1]}": [H("2/1", 1, 10)], "2|M|1": [H("2/1", 1, 10, "PHP")],
        "2|M|2": [POP], **adj_routes(2, ring[1]["adjs"]),
        f"3|U|{ADDR[4]}": [H("3/4", 4, 10)], "3|M|4": [H("3/4", 4, 10, "PHP")],
        f"3|U|{ADDR[2]}": [H("3/1", 1, 20), H("3/4", 4, 20)],
        "3|M|2": [H("3/1", 1, 20, "SWAP", [2]), H("3/4", 4, 20, "SWAP", [2])],
        f"3|U|{ADDR[1]}": [H("3/1", 1, 10)], "3|M|1": [H("3/1", 1, 10, "PHP")],
        "3|M|3": [POP], **adj_routes(3, ring[2]["adjs"]),
        f"4|U|{ADDR[3]}": [H("4/3", 3, 10)], "4|M|3": [H("4/3", 3, 10, "PHP")],
        f"4|U|{ADDR[2]}": [H("4/2", 2, 10)], "4|M|2": [H("4/2", 2, 10, "PHP")],
        f"4|U|{ADDR[1]}": [H("4/2", 2, 20), H("4/3", 3, 20)],
        "4|M|1": [H("4/2", 2, 20, "SWAP", [1]), H("4/3", 3, 20, "SWAP", [1])],
        "4|M|4": [POP], **adj_routes(4, ring[3]["adjs"])}
    e.update(extra or {})
    return e


fixtures.append(dict(
    name="decision_simple_ring_multipath_routes",
    source="openr/decision/tests/DecisionTest.cpp:2231-2365",
    steps=[dict(dbs=ring, expect_changes=ring_changes, checks=[
        route_map([1, 2, 3, 4], ring_pfx, expect_size=36, expect=_ring_full())])]))

# SimpleRingTopologyFixture.AttachedNodesTest (DecisionTest.cpp:3058-3108):
# the default route from nodes 1 and 4; attached nodes get none
_ring_dflt = dict(ring_pfx, **{"::/0": [["1", "ip", "ecmp", 0, None], ["4", "ip", "ecmp", 0, None]]})
fixtures.append(dict(
    name="decision_simple_ring_attached_nodes",
    source="openr/decision/tests/DecisionTest.cpp:3058-3108",
    steps=[dict(dbs=ring, expect_changes=ring_changes, checks=[
        route_map([1, 2, 3, 4], _ring_dflt, expect_size=38,
                  expect={"2|U|::/0": [H("2/1", 1, 10), H("2/4", 4, 10)],
                          "3|U|::/0": [H("3/1", 1, 10), H("3/4", 4, 10)]},
                  expect_absent=["1|U|::/0", "4|U|::/0"])])]))

# SimpleRingTopologyFixture.DuplicateMplsRoutes (DecisionTest.cpp:2174-2226):
# node 1 takes node 2's label 2; every node keeps exactly one route to label
# 2 (the reference counts the duplicate, :2195-2198). Which node keeps it is
# buildRouteDb's rule (SpfSolver.cpp:525-539: on a collision the node whose
# name sorts first keeps the label, whatever the iteration order): node 1.
# Then node 1 goes back to label 1: label 2 is node 2's again, nothing else
# is withdrawn (:2211-2225).
_r1dup = db(1, [dadj(1, 2), dadj(1, 3)], 2)
fixtures.append(dict(
    name="decision_simple_ring_duplicate_mpls_routes",
    source="openr/decision/tests/DecisionTest.cpp:2174-2226",
    steps=[
        dict(dbs=ring, expect_changes=ring_changes),
        dict(dbs=[_r1dup], expect_changes=[[False, False, True, None]], checks=[
            route_map([1, 2, 3, 4], ring_pfx,
                      expect_counts={"1": [3, 5], "2": [3, 5], "3": [3, 5], "4": [3, 5]},
                      expect={"1|M|2": [POP], "2|M|2": [H("2/1", 1, 10, "PHP")],
                              "3|M|2": [H("3/1", 1, 10, "PHP")],
                              "4|M|2": [H("4/2", 2, 20, "SWAP", [2]),
                                        H("4/3", 3, 20, "SWAP", [2])]},
                      expect_absent=["1|M|1", "2|M|1", "3|M|1", "4|M|1"])]),
        dict(dbs=[ring[0]], expect_changes=[[False, False, True, None]], checks=[
            route_map([1, 2, 3, 4], ring_pfx, expect_size=36, expect=_ring_full())]),
    ]))

# ParallelAdjRingTopologyFixture.MultiPathTest (DecisionTest.cpp:3711-3857):
# the same route map as ShortestPathTest (multipath is ignored)
fixtures.append(dict(
    name="decision_parallel_adj_ring_multipath_routes",
    source="openr/decision/tests/DecisionTest.cpp:3711-3857",
    steps=[dict(
        dbs=pr, expect_changes=[[False, None, None, None], [True, None, None, None],
                                [True, None, None, None], [True, None, None, None]],
        checks=[route_map([1, 2, 3, 4], ring_pfx, expect_size=44, expect={
            f"1|U|{ADDR[4]}": _p1_4, "1|M|4": _sw(_p1_4, 4),
            f"1|U|{ADDR[3]}": [H("3/1", 3, 11)], "1|M|3": [H("3/1", 3, 11, "PHP")],
            f"1|U|{ADDR[2]}": [H("2/1", 2, 11), H("2/2", 2, 11)],
            "1|M|2": _sw([H("2/1", 2, 11), H("2/2", 2, 11)], None),
            "1|M|1": [POP], **adj_routes(1, pr[0]["adjs"]),
            f"2|U|{ADDR[4]}": [H("4/1", 4, 11)], "2|M|4": [H("4/1", 4, 11, "PHP")],
            f"2|U|{ADDR[3]}": _p2_3, "2|M|3": _sw(_p2_3, 3),
            f"2|U|{ADDR[1]}": [H("1/1", 1, 11), H("1/2", 1, 11)],
            "2|M|1": _sw([H("1/1", 1, 11), H("1/2", 1, 11)], None),
            "2|M|2": [POP], **adj_routes(2, pr[1]["adjs"]),
            f"3|U|{ADDR[4]}": [H("4/1", 4, 11)], "3|M|4": [H("4/1", 4, 11, "PHP")],
            f"3|U|{ADDR[2]}": _p3_2, "3|M|2": _sw(_p3_2, 2),
            f"3|U|{ADDR[1]}": [H("1/1", 1, 11)], "3|M|1": [H("1/1", 1, 11, "PHP")],
            "3|M|3": [POP], **adj_routes(3, pr[2]["adjs"]),
            f"4|U|{ADDR[3]}": [H("3/1", 3, 11)], "4|M|3": [H("3/1", 3, 11, "PHP")],
            f"4|U|{ADDR[2]}": [H("2/1", 2, 11)], "4|M|2": [H("2/1", 2, 11, "PHP")],
            f"4|U|{ADDR[1]}": _p4_1, "4|M|1": _sw(_p4_1, 1),
            "4|M|4": [POP], **adj_routes(4, pr[3]["adjs"])})])]))

# SimpleRingTopologyFixture.IpToMplsLabelPrepend (DecisionTest.cpp:2374-2536),
# v6 / no prefix type: node 1's addr1 entry is SR_MPLS + SP_ECMP (:2403-2418).
# Case 1 (:2419-2437) whole; case 3's prepend label (:2463-2478) for nodes 1
# and 4 only -- the reference keeps case 2's minNexthop = 2 there, which
# removes the routes of nodes 2 and 3 (RIB policy, not restated). Case 4
# needs static MPLS routes (updateStaticMplsRoutes): not restated.
_pp = 10001
fixtures.append(dict(
    name="decision_ip_to_mpls_label_prepend",
    source="openr/decision/tests/DecisionTest.cpp:2374-2536",
    steps=[dict(dbs=ring, expect_changes=ring_changes, checks=[
        route_map([1, 2, 3, 4], {ADDR[1]: [["1", "sr_mpls", "ecmp", 0, None]]},
                  expect={f"2|U|{ADDR[1]}": [H("2/1", 1, 10)],
                          f"3|U|{ADDR[1]}": [H("3/1", 1, 10)],
                          f"4|U|{ADDR[1]}": [H("4/2", 2, 20, "PUSH", [1]),
                                             H("4/3", 3, 20, "PUSH", [1])]},
                  expect_absent=[f"1|U|{ADDR[1]}"]),
        route_map([1, 4], {ADDR[1]: [["1", "sr_mpls", "ecmp", 0, _pp]]},
                  expect={f"4|U|{ADDR[1]}": [H("4/2", 2, 20, "PUSH", [_pp, 1]),
                                             H("4/3", 3, 20, "PUSH", [_pp, 1])]},
                  expect_absent=[f"1|U|{ADDR[1]}"]),
    ])]))

# ConnectivityTest.CompatibilityNodeTest (DecisionTest.cpp:1564-1688):
# adjacencies of the "old" kind (labels 10000xx, metric 20 on 1-2)
_c12_1 = adj("2", "1/2", "2/1", 10, 1000021)
_c12_2 = adj("2", "1/2", "2/1", 20, 1000022)
_c13 = adj("3", "1/3", "3/1", 10, 1000031)
_c21 = adj("1", "2/1", "1/2", 10, 1000011)
_c23 = adj("3", "2/3", "3/2", 10, 100003)
_c32 = adj("2", "3/2", "2/3", 10, 100002)
_c31 = adj("1", "3/1", "1/3", 10, 1000011)
_cpx = loopbacks([1, 2, 3])
fixtures.append(dict(
    name="decision_connectivity_compatibility_node",
    source="openr/decision/tests/DecisionTest.cpp:1564-1688",
    steps=[
        dict(dbs=[db(2, [_c21, _c23], 2), db(3, [_c32, _c31], 3), db(1, [_c12_1], 1)],
             expect_changes=[[False, None, None, None], [True, None, None, None],
                             [True, None, None, None]]),
        dict(dbs=[db(1, [_c12_1, _c13], 1)], expect_changes=[[True, None, None, None]]),
        dict(dbs=[db(1, [_c12_2, _c13], 1)], expect_changes=[[True, None, None, None]],
             checks=[route_map([1, 2, 3], _cpx, expect_size=21, expect={
                 f"1|U|{ADDR[2]}": [H("1/2", 2, 20), H("1/3", 3, 20)],
                 f"1|U|{ADDR[3]}": [H("1/3", 3, 10)],
                 "1|M|2": [H("1/2", 2, 20, "PHP"), H("1/3", 3, 20, "SWAP", [2])],
                 "1|M|3": [H("1/3", 3, 10, "PHP")],
                 "1|M|1": [POP], **adj_routes(1, [_c12_2, _c13]),
                 f"2|U|{ADDR[3]}": [H("2/3", 3, 10)], f"2|U|{ADDR[1]}": [H("2/1", 1, 10)],
                 "2|M|1": [H("2/1", 1, 10, "PHP")], "2|M|3": [H("2/3", 3, 10, "PHP")],
                 f"3|U|{ADDR[2]}": [H("3/2", 2, 10)], f"3|U|{ADDR[1]}": [H("3/1", 1, 10)],
                 "3|M|1": [H("3/1", 1, 10, "PHP")], "3|M|2": [H("3/2", 2, 10, "PHP")],
                 "3|M|3": [POP], **adj_routes(3, [_c32, _c31])})]),
        dict(dbs=[db(1, [_c12_2], 0)], expect_changes=[[True, None, None, None]]),
        dict(dbs=[db(3, [_c32], 0)], expect_changes=[[False, None, None, None]]),
        dict(dbs=[db(1, [_c12_2, _c13], 0)], expect_changes=[[False, None, None, None]]),
    ]))

# DecisionTest.Ip2MplsRoutes (DecisionTest.cpp:4254-4550): SR_MPLS loopbacks
# of 1-3, the default route from 4 and 5, no adjacency labels; 15 unicast +
# 25 node-label routes
def _ia(other, ifn, oif, metric):
    return adj(str(other), ifn, oif, metric, 0)


_ip = [db(1, [_ia(2, "2/1", "1/1", 10), _ia(2, "2/2", "1/2", 10), _ia(3, "3/1", "1/1", 10)], 1),
       db(2, [_ia(1, "1/1", "2/1", 10), _ia(1, "1/2", "2/2", 10), _ia(4, "4/1", "2/1", 10),
              _ia(5, "5/1", "2/1", 10)], 2),
       db(3, [_ia(1, "1/1", "3/1", 10), _ia(4, "4/1", "3/1", 20), _ia(5, "5/1", "3/1", 10)], 3),
       db(4, [_ia(2, "2/1", "4/1", 10), _ia(3, "3/1", "4/1", 20)], 4),
       db(5, [_ia(2, "2/1", "5/1", 10), _ia(3, "3/1", "5/1", 10)], 5)]
_ipx = {ADDR[1]: [["1", "sr_mpls", "ecmp", 0, None]], ADDR[2]: [["2", "sr_mpls", "ecmp", 0, None]],
        ADDR[3]: [["3", "sr_mpls", "ecmp", 0, None]],
        "::/0": [["4", "sr_mpls", "ecmp", 0, None], ["5", "sr_mpls", "ecmp", 0, None]]}
fixtures.append(dict(
    name="decision_ip2mpls_routes",
    source="openr/decision/tests/DecisionTest.cpp:4254-4550",
    steps=[dict(
        dbs=_ip, expect_changes=[[False, None, None, None]] + [[True, None, None, None]] * 4,
        checks=[route_map([1, 2, 3, 4, 5], _ipx, expect_size=40, expect={
            "1|M|1": [POP],
            f"1|U|{ADDR[2]}": [H("2/2", 2, 10), H("2/1", 2, 10)],
            f"1|U|{ADDR[3]}": [H("3/1", 3, 10)],
            "1|U|::/0": [H("3/1", 3, 20, "PUSH", [5]), H("2/2", 2, 20, "PUSH", [4]),
                         H("2/2", 2, 20, "PUSH", [5]), H("2/1", 2, 20, "PUSH", [4]),
                         H("2/1", 2, 20, "PUSH", [5])],
            "1|M|2": [H("2/1", 2, 10, "PHP"), H("2/2", 2, 10, "PHP")],
            "1|M|3": [H("3/1", 3, 10, "PHP")],
            "1|M|4": [H("2/1", 2, 20, "SWAP", [4]), H("2/2", 2, 20, "SWAP", [4])],
            "1|M|5": [H("2/1", 2, 20, "SWAP", [5]), H("2/2", 2, 20, "SWAP", [5]),
                      H("3/1", 3, 20, "SWAP", [5])],
            "2|M|2": [POP],
            f"2|U|{ADDR[1]}": [H("1/1", 1, 10), H("1/2", 1, 10)],
            f"2|U|{ADDR[3]}": [H("1/1", 1, 20, "PUSH", [3]), H("1/2", 1, 20, "PUSH", [3]),
                               H("5/1", 5, 20, "PUSH", [3])],
            "2|U|::/0": [H("4/1", 4, 10), H("5/1", 5, 10)],
            "2|M|1": [H("1/1", 1, 10, "PHP"), H("1/2", 1, 10, "PHP")],
            "2|M|3": [H("1/1", 1, 20, "SWAP", [3]), H("1/2", 1, 20, "SWAP", [3]),
                      H("5/1", 5, 20, "SWAP", [3])],
            "2|M|4": [H("4/1", 4, 10, "PHP")], "2|M|5": [H("5/1", 5, 10, "PHP")],
            "3|M|3": [POP],
            f"3|U|{ADDR[1]}": [H("1/1", 1, 10)],
            f"3|U|{ADDR[2]}": [H("1/1", 1, 20, "PUSH", [2]), H("5/1", 5, 20, "PUSH", [2])],
            "3|U|::/0": [H("5/1", 5, 10)],
            "3|M|1": [H("1/1", 1, 10, "PHP")],
            "3|M|2": [H("1/1", 1, 20, "SWAP", [2]), H("5/1", 5, 20, "SWAP", [2])],
            "3|M|4": [H("4/1", 4, 20, "PHP")], "3|M|5": [H("5/1", 5, 10, "PHP")],
            "4|M|4": [POP],
            f"4|U|{ADDR[1]}": [H("2/1", 2, 20, "PUSH", [1])],
            f"4|U|{ADDR[2]}": [H("2/1", 2, 10)], f"4|U|{ADDR[3]}": [H("3/1", 3, 20)],
            "4|M|1": [H("2/1", 2, 20, "SWAP", [1])], "4|M|2": [H("2/1", 2, 10, "PHP")],
            "4|M|3": [H("3/1", 3, 20, "PHP")], "4|M|5": [H("2/1", 2, 20, "SWAP", [5])],
            "5|M|5": [POP],
            f"5|U|{ADDR[1]}": [H("2/1", 2, 20, "PUSH", [1]), H("3/1", 3, 20, "PUSH", [1])],
            f"5|U|{ADDR[2]}": [H("2/1", 2, 10)], f"5|U|{ADDR[3]}": [H("3/1", 3, 10)],
            "5|M|1": [H("2/1", 2, 20, "SWAP", [1]), H("3/1", 3, 20, "SWAP", [1])],
            "5|M|2": [H("2/1", 2, 10, "PHP")], "5|M|3": [H("3/1", 3, 10, "PHP")],
            "5|M|4": [H("2/1", 2, 20, "SWAP", [4])]})])]))

# LinkStateTest.pathAInPathB (LinkStateTest.cpp:211-254)
_l1, _l2, _l3 = "1%1/2|2%2/1", "2%2/3|3%3/2", "1%1/3|3%3/1"
fixtures.append(dict(
    name="linkstate_path_a_in_path_b",
    source="openr/decision/tests/LinkStateTest.cpp:211-254",
    steps=[dict(dbs=[], checks=[dict(kind="path_in", cases=[
        [[], [], True], [[], [], True],
        [[_l1], [], False], [[], [_l1], True],
        [[_l1], [_l1], True], [[_l1], [_l1], True],
        [[_l1, _l2], [_l1], False], [[_l1], [_l1, _l2], True],
        [[_l1, _l2, _l3], [_l1, _l2], False], [[_l1, _l2], [_l1, _l2, _l3], True],
        [[_l3, _l2], [_l1], False], [[_l1], [_l3, _l2], False],
    ])])]))


# Decision.BestRouteSelection (DecisionTest.cpp:1240-1384): SpfSolver with
# enableBestRouteSelection; 2 <-> 1 <-> 3 (adj12, adj13, adj21, adj31 of
# :46-106: metric 10); addr1 announced by 2 (DEFAULT) and 3 (BGP, no metric
# vector -- the type plays no part in best-route selection), createMetrics(pp,
# sp, d) (LsdbUtil.cpp:556-562). Entry = [node, fwd, algo, weight, prepend,
# area, minNexthop, (pp, sp, d), type].
_b1 = [db(1, [dadj(1, 2), dadj(1, 3)], 1), db(2, [dadj(2, 1)], 2), db(3, [dadj(3, 1)], 3)]
_bopt = dict(best_route_selection=True)


def _be(node, fwd, met, typ=None):
    return [str(node), fwd, "ecmp", 0, None, None, None, list(met), typ]


fixtures.append(dict(
    name="decision_best_route_selection",
    source="openr/decision/tests/DecisionTest.cpp:1240-1384",
    steps=[dict(dbs=_b1, checks=[
        # Case 1 (:1291-1320): node 1 ECMP towards {2, 3}; best routes {2, 3},
        # best node 2
        route_map([1], {ADDR[1]: [_be(2, "ip", (200, 0, 0)), _be(3, "ip", (200, 0, 0), "bgp")]},
                  opts=_bopt, expect_counts={"1": [1, None]},
                  expect={f"1|U|{ADDR[1]}": [H("1/2", 2, 10), H("1/3", 3, 10)]},
                  expect_best={f"1|{ADDR[1]}": ["2", ["2", "3"]]}),
        # Case 2 (:1322-1352): node 2's source preference 100 -> only node 2
        route_map([1], {ADDR[1]: [_be(2, "ip", (200, 100, 0)), _be(3, "ip", (200, 0, 0), "bgp")]},
                  opts=_bopt, expect_counts={"1": [1, None]},
                  expect={f"1|U|{ADDR[1]}": [H("1/2", 2, 10)]},
                  expect_best={f"1|{ADDR[1]}": ["2", ["2"]]}),
        # Case 3 (:1354-1383): the forwarding type comes from the best entry:
        # node 2 SR_MPLS (preferred), node 3 IP; from node 3: PUSH 2 via 1
        route_map([3], {ADDR[1]: [_be(2, "sr_mpls", (200, 100, 0)),
                                  _be(3, "ip", (200, 0, 0), "bgp")]},
                  opts=_bopt, expect_counts={"3": [1, None]},
                  expect={f"3|U|{ADDR[1]}": [H("3/1", 1, 20, "PUSH", [2])]}),
    ])]))

# EnableBestRouteSelectionFixture.PrefixWithMixedTypeRoutes
# (DecisionTest.cpp:7203-7290): 10.1.0.0/16 announced by 2 as BGP (with a
# metric vector, empty) and by 3 as RIB: skipped (decision.skipped_unicast_
# route) unless best-route selection is on.
_mix = {"10.1.0.0/16": [[ "2", "ip", "ecmp", 0, None, None, None, None, "bgpmv"],
                        ["3", "ip", "ecmp", 0, None, None, None, None, None]]}
fixtures.append(dict(
    name="decision_best_route_selection_mixed_types",
    source="openr/decision/tests/DecisionTest.cpp:7203-7290",
    steps=[dict(dbs=_b1, checks=[
        route_map([1], _mix, opts=dict(best_route_selection=False),
                  expect_counts={"1": [0, None]}, expect_absent=["1|U|10.1.0.0/16"]),
        route_map([1], _mix, opts=_bopt, expect_counts={"1": [1, None]}),
    ])]))


def main():
    for fx in fixtures:
        with open(os.path.join(HERE, fx["name"] + ".json"), "w") as f:
            json.dump(fx, f, indent=1, sort_keys=True)
    print(f"wrote {len(fixtures)} fixtures")


if __name__ == "__main__":
    main()
