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
from typing import Callable, Dict, List, Optional

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


def i32(m: int) -> int:
    """createNextHop's int32 metric (LsdbUtil.cpp:658-675): low 32 bits."""
    return ((m + 2 ** 31) % 2 ** 32) - 2 ** 31


def valid_label(lbl: int) -> bool:
    """isMplsLabelValid (MplsUtil.h:19-22)."""
    return (lbl & 0xfff00000) == 0 and lbl != 0


class RouteBuilder:
    """Test-side restatement of SpfSolver::buildRouteDb (SpfSolver.cpp:460-646)
    for one area, over any LinkState-like object plus the current adjacency
    databases (node labels, adjacency labels). Mirrors, line by line:
    createRouteForPrefix :197-458 (reachable announcers, drained filter
    :709-731, self-origination :333-337, forwarding type/algorithm = min over
    best entries LsdbUtil.cpp:379-413), selectBestPathsSpf :772-845,
    getNextHopsWithMetric :1043-1089, getNodeUcmpResult :1091-1161,
    getNextHopsThrift :1163-1285, selectBestPathsKsp2 :847-973.
    Next hop = (ifName, neighbor, metric i32, op, labels, weight)."""

    def __init__(self, ls, dbs: Dict[str, dict], ucmp: bool = False,
                 node_labels: bool = True, adj_labels: bool = True,
                 best_route_selection: bool = False, area: str = "0"):
        self.ls, self.dbs, self.ucmp = ls, dbs, ucmp
        self.node_labels, self.adj_labels = node_labels, adj_labels
        self.best_sel, self.area = best_route_selection, area
        self._spf = {}

    def spf(self, me):
        if me not in self._spf:
            self._spf[me] = self.ls.spf(me)
        return self._spf[me]

    def label(self, node) -> int:
        return self.dbs[node]["node_label"] if node in self.dbs else 0

    def adj_label(self, me, key) -> int:
        ifn, other = if_from(key, me), other_of(key, me)
        for a in self.dbs[me]["adjs"]:
            if a["if_name"] == ifn and a["other"] == other:
                return a["label"]
        return 0

    def with_metric(self, me, dsts, per_dst):
        res = self.spf(me)
        shortest, closest = None, []
        for d in dsts:
            if d not in res:
                continue
            m = res[d][0]
            if shortest is None or m < shortest:
                shortest, closest = m, []
            if m == shortest:
                closest.append(d)
        via = {}
        for d in closest:
            for nh in res[d][1]:
                via[(nh, d if per_dst else "")] = shortest - res[nh][0]
        return shortest, via

    def next_hops(self, me, dsts, per_dst, shortest, via, swap=None, entries=None,
                  ucmp_hops=None):
        out = set()
        dset = set(dsts)
        for key, metric, up in self.ls.links(me):
            nbr = other_of(key, me)
            for dst in (sorted(dset) if per_dst else [""]):
                if (nbr, dst) not in via or not up:
                    continue
                if dst and nbr in dset and nbr != dst:
                    continue
                over = metric + via[(nbr, dst)]
                if over != shortest:
                    continue
                op, labels = "", ()
                if swap is not None:
                    op, labels = ("PHP", ()) if nbr in dset else ("SWAP", (swap,))
                if dst:
                    push, ok = [], True
                    pl = entries[dst][4]
                    if pl is not None:
                        push.append(pl)
                        ok &= valid_label(pl)
                    if dst != nbr:
                        push.append(self.label(dst))
                        ok &= valid_label(push[-1])
                    if not ok:
                        continue
                    if push:
                        op, labels = "PUSH", tuple(push)
                ifn = if_from(key, me)
                w = 0
                if ucmp_hops is not None and ifn in ucmp_hops:
                    w = ucmp_hops[ifn][1]
                out.add((ifn, nbr, i32(over), op, labels, w))
        return out

    def ksp2(self, me, best, entries):
        paths = []
        for n in best:
            if n != me:
                paths += self.ls.kth_paths(me, n, 1)
        first = len(paths)
        for n in best:
            for p in self.ls.kth_paths(me, n, 2):
                if not any(path_in(paths[i], p) for i in range(first)):
                    paths.append(p)
        out = set()
        for p in paths:
            cost, node, lbl, ok = 0, me, [], True
            for key in p:
                cost += next(m for k, m, _ in self.ls.links(node) if k == key)
                node = other_of(key, node)
                lbl.insert(0, self.label(node))
                ok &= valid_label(lbl[0])
            if not ok:
                continue
            lbl.pop()
            if node in entries and entries[node][4] is not None:
                lbl.insert(0, entries[node][4])
            out.add((if_from(p[0], me), other_of(p[0], me), i32(cost),
                     "PUSH" if lbl else "", tuple(lbl), 0))
        return out

    def prefix_route(self, me, ents):
        res = self.spf(me)
        entries = {e[0]: e for e in ents if e[0] in res}
        if not entries:
            return None
        self_prepend = entries[me][4] is not None if me in entries else True
        # selectBestRoutes (SpfSolver.cpp:650-674)
        if self.best_sel:
            # selectRoutes(SHORTEST_DISTANCE) (LsdbUtil.cpp:772-793,837-880):
            # highest (path_preference, source_preference), then lowest distance
            def met(n):
                e = entries[n]
                return tuple(e[7]) if len(e) > 7 and e[7] is not None else (0, 0, 0)
            top = max(met(n)[:2] for n in entries)
            tied = [n for n in entries if met(n)[:2] == top]
            dmin = min(met(n)[2] for n in tied)
            sel = sorted(n for n in tied if met(n)[2] == dmin)
            best_node = me if me in sel else sel[0]  # selectBestNodeArea (:758-769)
        else:
            typ = {n: (e[8] if len(e) > 8 else None) for n, e in entries.items()}
            if any(typ.values()) and (not all(typ.values()) or "bgp" in typ.values()):
                return None  # mixed BGP / other, or BGP without mv (:282-300)
            assert not any(typ.values()), "BGP metric-vector selection is not restated"
            sel = sorted(entries)
            best_node = sel[0]
        # maybeFilterDrainedNodes (:709-731): the best entry stays as selected
        best = sorted(n for n in sel if not self.ls.is_overloaded(n)) or sel
        self.last_best = ((best_node, self.area), tuple((n, self.area) for n in best))
        if me in best and not self_prepend:
            return None
        fwd = min({"ip": 0, "sr_mpls": 1}[entries[n][1]] for n in best)
        algo = min({"ecmp": 0, "ksp2": 1, "ucmp_adj": 2, "ucmp_prefix": 3}[entries[n][2]]
                   for n in best)
        shortest, weight = 2 ** 64 - 1, None
        if algo == 1:
            nhs = self.ksp2(me, best, entries) if fwd == 1 else set()
        else:
            per_dst = fwd == 1
            filt = [n for n in best
                    if not (n == me and per_dst and entries[me][4] is not None)]
            shortest, via = self.with_metric(me, filt, per_dst)
            if shortest is None:
                shortest = 2 ** 64 - 1
            nhs = set()
            if via:
                hops = None
                if self.ucmp and algo in (2, 3):
                    leaves, ok = {}, True
                    for n in best:
                        if n not in res or res[n][0] != shortest:
                            continue
                        if not entries[n][3]:
                            ok = False
                            break
                        leaves[n] = entries[n][3]
                    if ok:
                        u = self.ls.ucmp(me, leaves, "adj" if algo == 2 else "prefix")
                        if me in u:
                            weight, hops = u[me]
                nhs = self.next_hops(me, best, per_dst, shortest, via, entries=entries,
                                     ucmp_hops=hops)
        if not nhs:
            return None
        return (shortest % 2 ** 32, weight), nhs

    def build(self, me, prefixes):
        if me not in self.dbs:
            return None
        out = {"routes": {}}
        for p, ents in prefixes.items():
            r = self.prefix_route(me, ents)
            if r is not None:
                out["routes"][p] = r[0]
                out[("U", p)] = r[1]
                if self.best_sel:
                    out.setdefault("best", {})[p] = self.last_best
        if self.node_labels:
            label_to = {}
            for node in sorted(self.dbs):
                top = self.dbs[node]["node_label"]
                if top == 0 or not valid_label(top):
                    continue
                if top in label_to and label_to[top][0] < node:
                    continue
                if node == me:
                    label_to[top] = (me, {("", "", 0, "POP", (), 0)})
                    continue
                shortest, via = self.with_metric(me, [node], False)
                if not via:
                    continue
                label_to[top] = (node, self.next_hops(me, [node], False, shortest, via,
                                                      swap=top))
            for top, (_, nhs) in label_to.items():
                out[("M", str(top))] = nhs
        if self.adj_labels:
            for key, metric, _ in self.ls.links(me):
                top = self.adj_label(me, key)
                if top == 0 or not valid_label(top):
                    continue
                assert ("M", str(top)) not in out, f"duplicate MPLS label {top}"
                out[("M", str(top))] = {(if_from(key, me), other_of(key, me), i32(metric),
                                         "PHP", (), 0)}
        return out


def _hop_set(expect):
    return {(h[0], h[1], h[2], h[3], tuple(h[4]), h[5]) for h in expect}


def check_route_map(c, dbs_of: Callable[[str], dict], where: str):
    """Assert one route_map check against {node: route db | None}."""
    n_routes = 0
    for node in c["nodes"]:
        db = dbs_of(node)
        exp = c.get("expect_counts", {}).get(node, "skip")
        if exp is None:
            assert db is None, f"{where}: {node} expected no route db"
        if db is None:
            assert exp in (None, "skip"), f"{where}: {node} has no route db"
            continue
        n_u = sum(1 for k in db if k[0] == "U")
        n_m = sum(1 for k in db if k[0] == "M")
        n_routes += n_u + n_m
        if exp not in (None, "skip"):
            if exp[0] is not None:
                assert n_u == exp[0], f"{where}: {node} unicast {n_u} != {exp[0]}"
            if exp[1] is not None:
                assert n_m == exp[1], f"{where}: {node} mpls {n_m} != {exp[1]}"
    if "expect_size" in c:
        assert n_routes == c["expect_size"], f"{where}: route map size {n_routes}"
    for k, hops in c.get("expect", {}).items():
        node, kind, key = k.split("|", 2)
        got = (dbs_of(node) or {}).get((kind, key))
        assert got == _hop_set(hops), f"{where}: {k} {sorted(got or [])}"
    for k in c.get("expect_absent", []):
        node, kind, key = k.split("|", 2)
        assert (kind, key) not in (dbs_of(node) or {}), f"{where}: {k} present"
    for k, m in c.get("expect_metric", {}).items():
        node, kind, key = k.split("|", 2)
        got = dbs_of(node)[(kind, key)]
        assert {h[2] for h in got} == {m}, f"{where}: {k} metrics {got}"
    for k, (b, sel) in c.get("expect_best", {}).items():
        node, key = k.split("|", 1)  # bestRoutesCache_: best node, every selected node
        got = dbs_of(node)["best"][key]
        assert got[0][0] == b and sorted(x[0] for x in got[1]) == sorted(sel), \
            f"{where}: {k} best {got}"
    for k, w in c.get("expect_weight", {}).items():
        node, key = k.split("|", 1)
        assert dbs_of(node)["routes"][key][1] == w, \
            f"{where}: {k} weight {dbs_of(node)['routes'][key]}"


def _as_set(expect):
    if expect is None:
        return None
    return {(e[0], e[1], tuple(e[2])) for e in expect}


SPF_KINDS = {"spf_runs", "ecmp", "ecmp_all", "ksp2", "ksp2_all", "kth_paths",
             "kth_paths_edge_disjoint", "reachable", "grid_manhattan", "ucmp", "route_map"}


def run_fixture(fx: dict, make_ls, check_changes: bool = True, spf: bool = True) -> int:
    """Apply every step and assert every check. Returns #checks evaluated.
    spf=False evaluates only ingest-level checks (no SPF needed)."""
    ls = make_ls()
    labels: Dict[str, int] = {}
    cur: Dict[str, dict] = {}  # the adjacency databases the link state holds
    n_checks = 0
    for si, step in enumerate(fx["steps"]):
        st = stream_of(step["dbs"])
        changes = ls.apply(st)
        for d in step["dbs"]:
            labels[d["name"]] = d["node_label"]
            if d["delete"]:
                cur.pop(d["name"], None)
            else:
                cur[d["name"]] = d
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
            elif k == "route_map":
                opts = c.get("opts", {})
                rb = RouteBuilder(ls, cur, **opts)
                mine = {n: rb.build(n, c.get("prefixes", {})) for n in c["nodes"]}
                check_route_map(c, mine.get, where)
                if hasattr(ls, "route_dbs"):  # the product's C++ SpfSolver port
                    prod = ls.route_dbs(c["nodes"], c.get("prefixes", {}), **opts)
                    check_route_map(c, prod.get, where + " C++")
                    assert prod == mine, f"{where}: C++ route dbs differ from restatement"
            elif k == "path_in":
                for a, b, want in c["cases"]:
                    assert path_in(a, b) == want, f"{where}: {a} in {b}"
                    if hasattr(ls, "path_a_in_b"):
                        assert ls.path_a_in_b(a, b) == want, f"{where}: C++ {a} in {b}"
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
