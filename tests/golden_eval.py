"""Evaluate tests/golden/*.json fixtures against any LinkState-like object.

A LinkState-like object (the CPU oracle, or the product's GPU-backed
openr_amd.LinkState) provides::

    apply(stream) -> [(topo, attrs, label, n_added), ...]
    spf(root, use_link_metric=True) -> {name: (metric, nexthops, pathlinks)}
    kth_paths(src, dst, k) -> [[link_key, ...], ...]
    links(node) -> [(link_key, metric_from_node, up), ...]
    is_overloaded(node) -> bool
    spf_runs -> int

Route sets are rebuilt from those results exactly as the reference's
SpfSolver does for a node-loopback prefix announced by a single node:
SP_ECMP  = getNextHopsWithMetric + getNextHopsThrift (SpfSolver.cpp:1043-1285,
           perDestination=false);
KSP2_ED_ECMP = selectBestPathsKsp2 (SpfSolver.cpp:847-973).
"""
from __future__ import annotations

import glob
import json
import os
from typing import Dict, List, Optional

from openr_amd.adjdb import AdjDb, AdjDbStream, Adjacency

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_fixtures() -> List[dict]:
    out = []
    for p in sorted(glob.glob(os.path.join(GOLDEN_DIR, "*.json"))):
        with open(p) as f:
            out.append(json.load(f))
    return out


def stream_of(dbs: List[dict]) -> AdjDbStream:
    return AdjDbStream.from_dbs(
        AdjDb(d["name"], [Adjacency(**a) for a in d["adjs"]], d["node_label"],
              d["overloaded"], d["delete"]) for d in dbs)


def split_key(key: str):
    a, b = key.split("|")
    na, ia = a.split("%", 1)
    nb, ib = b.split("%", 1)
    return (na, ia), (nb, ib)


def if_from(key: str, node: str) -> str:
    (na, ia), (nb, ib) = split_key(key)
    return ia if na == node else ib


def other_of(key: str, node: str) -> str:
    (na, _), (nb, _) = split_key(key)
    return nb if na == node else na


def ecmp_routes(ls, src: str, dst: str) -> Optional[set]:
    if src == dst:
        return None
    res = ls.spf(src)
    if dst not in res:
        return None
    shortest = res[dst][0]
    nh_nodes = {nh: shortest - res[nh][0] for nh in res[dst][1]}
    out = set()
    for key, metric, up in ls.links(src):
        nb = other_of(key, src)
        if nb not in nh_nodes or not up:
            continue
        d = metric + nh_nodes[nb]
        if d != shortest:
            continue
        out.add((if_from(key, src), d, ()))
    return out or None


def path_in(a: List[str], b: List[str]) -> bool:
    """LinkState::pathAInPathB (LinkState.h:477-492)."""
    if len(a) > len(b):
        return False
    for i in range(len(b) - len(a) + 1):
        if b[i:i + len(a)] == a:
            return True
    return False


def ksp2_routes(ls, src: str, dst: str, labels: Dict[str, int],
                metrics: Dict[tuple, int]) -> Optional[set]:
    if src == dst:
        return None
    paths = [p for p in ls.kth_paths(src, dst, 1)]
    first = len(paths)
    for p in ls.kth_paths(src, dst, 2):
        if not any(path_in(paths[i], p) for i in range(first)):
            paths.append(p)
    out = set()
    for p in paths:
        cost, node, lbl = 0, src, []
        for key in p:
            cost += metrics[(key, node)]
            node = other_of(key, node)
            lbl.insert(0, labels[node])
        lbl.pop()  # PHP: drop the first hop's label
        out.add((if_from(p[0], src), cost, tuple(lbl)))
    return out or None


def _as_set(expect):
    if expect is None:
        return None
    return {(e[0], e[1], tuple(e[2])) for e in expect}


SPF_KINDS = {"spf_runs", "ecmp", "ecmp_all", "ksp2", "ksp2_all", "kth_paths",
             "kth_paths_edge_disjoint", "reachable", "grid_manhattan", "ucmp"}


def run_fixture(fx: dict, make_ls, check_changes: bool = True, spf: bool = True) -> int:
    """Apply every step and assert every check. Returns #checks evaluated.
    spf=False evaluates only ingest-level checks (no SPF needed)."""
    ls = make_ls()
    labels: Dict[str, int] = {}
    n_checks = 0
    for si, step in enumerate(fx["steps"]):
        st = stream_of(step["dbs"])
        changes = ls.apply(st)
        for d in step["dbs"]:
            labels[d["name"]] = d["node_label"]
        if check_changes and "expect_changes" in step:
            for got, exp in zip(changes, step["expect_changes"]):
                for g, e, what in zip(got, exp, ("topology", "attrs", "label", "added")):
                    if e is not None:
                        assert g == e, f"{fx['name']} step {si}: {what} {g} != {e}"
                        n_checks += 1
        metrics = {}
        nodes = {d["name"] for s in fx["steps"][: si + 1] for d in s["dbs"]}
        for nd in nodes:
            for key, m, _ in ls.links(nd):
                metrics[(key, nd)] = m
        for c in step.get("checks", []):
            k = c["kind"]
            if not spf and k in SPF_KINDS:
                continue
            where = f"{fx['name']} step {si} {c}"
            if k == "links":
                got = sorted(key for key, _, _ in ls.links(c["node"]))
                assert got == sorted(c["expect"]), f"{where}: {got}"
            elif k == "overloaded":
                assert ls.is_overloaded(c["node"]) == c["expect"], where
            elif k == "spf_runs":
                assert ls.spf_runs == c["expect"], f"{where}: spf_runs={ls.spf_runs}"
            elif k == "ecmp":
                assert ecmp_routes(ls, c["src"], c["dst"]) == _as_set(c["expect"]), \
                    f"{where}: {ecmp_routes(ls, c['src'], c['dst'])}"
                if hasattr(ls, "route"):  # the product's C++ SpfSolver port
                    got = ls.route(c["src"], [c["dst"]], "ecmp")
                    assert got == _as_set(c["expect"]), f"{where}: C++ {got}"
            elif k == "ecmp_all":
                for a in c["nodes"]:
                    for b in c["nodes"]:
                        ecmp_routes(ls, a, b)
            elif k == "ksp2":
                got = ksp2_routes(ls, c["src"], c["dst"], labels, metrics)
                assert got == _as_set(c["expect"]), f"{where}: {got}"
                if hasattr(ls, "route"):  # the product's C++ SpfSolver port
                    got = ls.route(c["src"], [c["dst"]], "ksp2")
                    assert got == _as_set(c["expect"]), f"{where}: C++ {got}"
            elif k == "ksp2_all":
                for a in c["nodes"]:
                    for b in c["nodes"]:
                        ksp2_routes(ls, a, b, labels, metrics)
            elif k == "kth_paths":
                paths = ls.kth_paths(c["src"], c["dst"], c["k"])
                if "expect_sizes" in c:
                    assert [len(p) for p in paths] == c["expect_sizes"], f"{where}: {paths}"
                if "expect_sizes_unordered" in c:
                    assert sorted(len(p) for p in paths) == sorted(c["expect_sizes_unordered"]), where
                if "expect_first_link_metric_from_src" in c:
                    assert metrics[(paths[0][0], c["src"])] == c["expect_first_link_metric_from_src"]
                if "expect_path_cost" in c:
                    for p in paths:
                        cost, node = 0, c["src"]
                        for key in p:
                            cost += metrics[(key, node)]
                            node = other_of(key, node)
                        assert cost == c["expect_path_cost"], where
            elif k == "kth_paths_edge_disjoint":
                seen = set()
                for kk in c["ks"]:
                    for p in ls.kth_paths(c["src"], c["dst"], kk):
                        for key in p:
                            assert key not in seen, where
                            seen.add(key)
            elif k == "reachable":
                assert (c["dst"] in ls.spf(c["src"])) == c["expect"], where
            elif k == "ucmp":
                got = ls.ucmp(c["root"], c["leaves"], c["algo"])
                if "expect_size" in c:
                    assert len(got) == c["expect_size"], f"{where}: {sorted(got)}"
                for node, e in c["expect"].items():
                    w, hops = got[node]
                    assert w == e["weight"], f"{where}: {node} weight {w}"
                    assert {i: hw for i, (_, hw) in hops.items()} == e["hops"], \
                        f"{where}: {node} hops {hops}"
            elif k == "grid_manhattan":
                n = c["n"]
                for s in range(n * n):
                    res = ls.spf(str(s))
                    assert len(res) == n * n, where
                    for t in range(n * n):
                        want = abs(s % n - t % n) + abs(s // n - t // n)
                        assert res[str(t)][0] == want, f"{where}: {s}->{t}"
            else:
                raise AssertionError(f"unknown check {k}")
            n_checks += 1
    return n_checks


class ProductLS:
    """Adapter: the product (GPU-backed) openr_amd.linkstate.LinkState."""

    def __new__(cls):
        from openr_amd.linkstate import LinkState
        return LinkState()


class OracleLS:
    """Adapter: oracle.Oracle -> LinkState-like (test side)."""

    def __init__(self):
        from oracle import Oracle, parse_spf_text
        self._o = Oracle()
        self._parse = parse_spf_text

    def apply(self, stream):
        return self._o.apply(stream)

    def spf(self, root, use_link_metric=True):
        return self._parse(self._o.spf_text(root, use_link_metric))

    def kth_paths(self, src, dst, k):
        return self._o.kth_paths(src, dst, k)

    def links(self, node):
        out = []
        for ln in self._o.links_text(node).splitlines():
            key, m, up = ln.split("\t")
            out.append((key, int(m), up == "1"))
        return out

    def is_overloaded(self, node):
        return self._o.is_overloaded(node)

    def ucmp(self, root, leaves, algo):
        return self._o.ucmp(root, leaves, algo)

    @property
    def spf_runs(self):
        return self._o.spf_runs
