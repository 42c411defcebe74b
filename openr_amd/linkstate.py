"""Python face of the GPU-backed LinkState mirror (libopenr_decision).

Method names follow openr/decision/LinkState.h (getSpfResult, getKthPaths,
getMetricFromAToB, linksFromNode, isNodeOverloaded, updateAdjacencyDatabase,
deleteAdjacencyDatabase); the snake_case helpers below are what the parity
tests drive.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import _native as N
from .adjdb import AdjDbStream, change_array, changes_to_list


class LinkStateError(RuntimeError):
    pass


def parse_ucmp_text(t: str) -> Dict[str, Tuple[int, Dict[str, Tuple[str, int]]]]:
    """odl/orc UCMP text -> {node: (advertised weight, {iface: (next hop, weight)})}."""
    out = {}
    for ln in t.splitlines():
        node, w, hops = ln.split("\t")
        hp = {}
        for h in filter(None, hops.split(",")):
            iface, rest = h.split("=", 1)
            nh, hw = rest.rsplit(":", 1)
            hp[iface] = (nh, int(hw))
        out[node] = (int(w), hp)
    return out


UCMP_ALGOS = {"adj": 2, "prefix": 3}  # SP_UCMP_{ADJ,PREFIX}_WEIGHT_PROPAGATION

# odl_route_db_bin records (include/openr_decision.h)
RDB_MAGIC = 0x4244524F
RDB_HEADER = np.dtype([("magic", "<u4"), ("version", "<u4"), ("bytes", "<u8"),
                       ("n_nodes", "<u4"), ("n_routes", "<u4"), ("n_nhs", "<u4"),
                       ("n_labels", "<u4"), ("off_nodes", "<u8"), ("off_routes", "<u8"),
                       ("off_nhs", "<u8"), ("off_labels", "<u8"), ("off_strings", "<u8"),
                       ("str_bytes", "<u8")])
RDB_NODE = np.dtype([("name", "<u4"), ("found", "<u4"), ("first_route", "<u4"),
                     ("n_unicast", "<u4"), ("n_mpls", "<u4"), ("pad", "<u4")])
RDB_ROUTE = np.dtype([("kind", "<u4"), ("key", "<u4"), ("igp_cost", "<u4"),
                      ("has_weight", "<u4"), ("ucmp_weight", "<i8"), ("first_nh", "<u4"),
                      ("n_nh", "<u4")])
RDB_NH = np.dtype([("if_name", "<u4"), ("neighbor", "<u4"), ("metric", "<i4"),
                   ("weight", "<i4"), ("op", "<u4"), ("first_label", "<u4"),
                   ("n_labels", "<u4"), ("pad", "<u4")])
_OPS = {0: "", 1: "PHP", 2: "SWAP", 3: "PUSH", 4: "POP"}


def decode_route_db_bin(buf: bytes):
    """odl_route_db_bin buffer -> route_dbs' dict (same shape as the text)."""
    hd = np.frombuffer(buf, RDB_HEADER, 1)[0]
    if int(hd["magic"]) != RDB_MAGIC or int(hd["version"]) != 1 or int(hd["bytes"]) != len(buf):
        raise ValueError("not an odl route-db buffer")
    nodes = np.frombuffer(buf, RDB_NODE, int(hd["n_nodes"]), int(hd["off_nodes"]))
    routes = np.frombuffer(buf, RDB_ROUTE, int(hd["n_routes"]), int(hd["off_routes"]))
    nhs = np.frombuffer(buf, RDB_NH, int(hd["n_nhs"]), int(hd["off_nhs"]))
    labels = np.frombuffer(buf, "<i4", int(hd["n_labels"]), int(hd["off_labels"])).tolist()
    so = int(hd["off_strings"])
    strs = buf[so: so + int(hd["str_bytes"])]
    cache = {}

    def sget(o):
        o = int(o)
        v = cache.get(o)
        if v is None:
            v = cache[o] = strs[o: strs.index(b"\0", o)].decode()
        return v

    out = {}
    for nd in nodes:
        me = sget(nd["name"])
        if not nd["found"]:
            out[me] = None
            continue
        db = {"routes": {}}
        r0 = int(nd["first_route"])
        for r in routes[r0: r0 + int(nd["n_unicast"]) + int(nd["n_mpls"])]:
            if r["kind"] == 0:
                key = sget(r["key"])
                db["routes"][key] = (int(r["igp_cost"]),
                                     int(r["ucmp_weight"]) if r["has_weight"] else None)
                kk = ("U", key)
            else:
                kk = ("M", str(int(np.int32(np.uint32(r["key"])))))
            f0 = int(r["first_nh"])
            if r["n_nh"]:
                db[kk] = {(sget(x["if_name"]), sget(x["neighbor"]), int(x["metric"]),
                           _OPS[int(x["op"])],
                           tuple(labels[int(x["first_label"]): int(x["first_label"]) + int(x["n_labels"])]),
                           int(x["weight"]))
                          for x in nhs[f0: f0 + int(r["n_nh"])]}
        out[me] = db
    return out


def _parse_spf(t: str) -> Dict[str, Tuple[int, tuple, tuple]]:
    out = {}
    for ln in t.splitlines():
        name, metric, nh, pl = ln.split("\t")
        out[name] = (int(metric), tuple(x for x in nh.split(",") if x),
                     tuple(x for x in pl.split(";") if x))
    return out


_FWDS = {"ip": 0, "sr_mpls": 1}
_ALGOS = {"ecmp": 0, "ksp2": 1, "ucmp_adj": 2, "ucmp_prefix": 3}
_TXT_OPS = {"0": "", "1": "PHP", "2": "SWAP", "3": "PUSH", "4": "POP"}


def _prefix_lines(prefixes) -> List[str]:
    """{prefix: [(node, fwd, algo, weight, prepend[, area[, min_nexthop[,
    metrics[, type]]]])]} -> the text ABI's
    "prefix\tnode:fwd:algo:weight:prepend[%pp/sp/d][!type][@area][#n],..."
    lines (metrics = (path_preference, source_preference, distance), type
    None | "bgp" | "bgpmv")"""
    lines = []
    for p, ents in prefixes.items():
        es = []
        for ent in ents:
            node, fwd, algo, weight, prepend = ent[:5]
            area = ent[5] if len(ent) > 5 else None
            mn = ent[6] if len(ent) > 6 else None
            met = ent[7] if len(ent) > 7 else None
            typ = ent[8] if len(ent) > 8 else None
            x = (f"{node}:{_FWDS[fwd]}:{_ALGOS[algo]}:{int(weight)}:"
                 f"{'' if prepend is None else int(prepend)}")
            if met is not None:
                x += "%" + "/".join(str(int(v)) for v in met)
            if typ:
                x += f"!{typ}"
            if area:
                x += f"@{area}"
            if mn is not None:
                x += f"#{int(mn)}"
            es.append(x)
        lines.append(f"{p}\t{','.join(es)}")
    return lines


def _parse_route_text(t: str, mes, with_area: bool):
    out = {me: {"routes": {}} for me in mes}
    for ln in t.splitlines():
        f = ln.split("\t")
        me, kind = f[0], f[1]
        if kind == "NONE":
            out[me] = None
        elif kind == "R":
            out[me]["routes"][f[2]] = (int(f[3]), None if f[4] == "-" else int(f[4]))
            if len(f) > 6:  # best-route selection on: (best, selected) as (node, area)
                sel = tuple(tuple(x.rsplit("@", 1)) for x in f[6].split(",") if x)
                out[me].setdefault("best", {})[f[2]] = (tuple(f[5].rsplit("@", 1)), sel)
        else:
            key, ifn, nbr, metric, op, labels, w = f[2:9]
            nh = (ifn, nbr, int(metric), _TXT_OPS[op], tuple(int(x) for x in labels.split(",") if x),
                  int(w))
            if with_area:
                nh += (f[9],)
            out[me].setdefault((kind, key), set()).add(nh)
    return out


def route_dbs_multi(areas: Sequence["LinkState"], mes: Sequence[str], prefixes,
                    node_labels: bool = True, adj_labels: bool = True, ucmp: bool = False,
                    best_route_selection: bool = False):
    """SpfSolver::buildRouteDb over several areas (odl_route_db_multi_text):
    one LinkState per area; prefix entries may carry (.., area, min_nexthop).
    Same result shape as LinkState.route_dbs(binary=False) with the next
    hop's area as a 7th tuple field."""
    L = N.decision()
    hs = (C.c_void_p * len(areas))(*[a._h for a in areas])
    lines = _prefix_lines(prefixes)
    flags = int(node_labels) | (2 if adj_labels else 0) | (4 if ucmp else 0) | \
        (8 if best_route_selection else 0)
    p = L.odl_route_db_multi_text(hs, len(areas), "\n".join(mes).encode(), len(mes),
                                  "\n".join(lines).encode(), len(lines), flags)
    if not p:
        raise LinkStateError(areas[0]._err())
    return _parse_route_text(areas[0]._take(p), mes, with_area=True)


class LinkState:
    """odl::LinkState over the MI355X SPF engine (device `device`)."""

    def __init__(self, area: str = "0", device: int = 0, stream: Optional[AdjDbStream] = None,
                 devices: Optional[Sequence[int]] = None):
        self._L = N.decision()
        h = C.c_void_p()
        if devices is not None and len(devices) > 1:
            devs = np.ascontiguousarray(devices, np.int32)
            rc = self._L.odl_create_multi(area.encode(), devs.ctypes.data, devs.size, C.byref(h))
        else:
            rc = self._L.odl_create(area.encode(), device if devices is None else devices[0],
                                    C.byref(h))
        if rc != 0:
            raise LinkStateError("odl_create failed")
        self._h = h
        if stream is not None:
            self.apply(stream)

    def __del__(self):
        if getattr(self, "_h", None):
            self._L.odl_destroy(self._h)
            self._h = None

    # ------------------------------------------------------------ plumbing
    def _err(self) -> str:
        return self._L.odl_last_error(self._h).decode()

    def _take(self, p) -> str:
        if not p:
            raise LinkStateError(self._err())
        s = C.cast(p, C.c_char_p).value.decode()
        self._L.odl_free(p)
        return s

    # ------------------------------------------------------------ ingest
    def apply(self, stream: AdjDbStream, first: int = 0, count: Optional[int] = None,
              hold_up_ttl: int = 0, hold_down_ttl: int = 0):
        """updateAdjacencyDatabase per record (LinkState.cpp:584-726), with its
        hold TTLs (0: Decision's own call, Decision.cpp:756)."""
        count = stream.n_dbs - first if count is None else count
        ch = change_array(count)
        if hold_up_ttl or hold_down_ttl:
            rc = self._L.odl_apply_hold(self._h, C.addressof(stream.struct), first, count,
                                        C.addressof(ch), hold_up_ttl, hold_down_ttl)
        else:
            rc = self._L.odl_apply(self._h, C.addressof(stream.struct), first, count,
                                   C.addressof(ch))
        if rc != 0:
            raise LinkStateError(self._err())
        return changes_to_list(ch, count)

    def decrement_holds(self) -> bool:
        """LinkState::decrementHolds (LinkState.cpp:520-535): True when a hold
        expired (topology changed)."""
        rc = self._L.odl_decrement_holds(self._h)
        if rc < 0:
            raise LinkStateError(self._err())
        return bool(rc)

    decrementHolds = decrement_holds

    def has_holds(self) -> bool:
        return self._L.odl_has_holds(self._h) == 1

    hasHolds = has_holds

    updateAdjacencyDatabases = apply

    # ------------------------------------------------------------ queries
    def spf_text(self, root: str, use_link_metric: bool = True) -> str:
        return self._take(self._L.odl_spf_text(self._h, root.encode(), int(use_link_metric)))

    def spf(self, root: str, use_link_metric: bool = True):
        return _parse_spf(self.spf_text(root, use_link_metric))

    getSpfResult = spf

    def kth_paths(self, src: str, dst: str, k: int) -> List[List[str]]:
        t = self._take(self._L.odl_kth_paths_text(self._h, src.encode(), dst.encode(), k))
        return [ln.split(",") for ln in t.splitlines()]

    getKthPaths = kth_paths

    def ksp2_text(self, src: str, dsts: Sequence[str]) -> str:
        return self._take(self._L.odl_ksp2_text(self._h, src.encode(),
                                                "\n".join(dsts).encode(), len(dsts)))

    def route(self, me: str, announcers: Sequence[str], algo: str = "ecmp"):
        """Route next-hops built in C++ (odl::SpfSolver): algo 'ecmp',
        'ksp2' or 'label'. Returns a set of (ifName, metric, labels)."""
        code = {"ecmp": 0, "ksp2": 1, "label": 2}[algo]
        t = self._take(self._L.odl_route_text(self._h, me.encode(),
                                              "\n".join(announcers).encode(),
                                              len(announcers), code))
        out = set()
        for ln in t.splitlines():
            ifn, nbr, metric, op, labels = ln.split("\t")
            out.add((ifn, int(metric), tuple(int(x) for x in labels.split(",") if x)))
        return out or None

    def route_dbs(self, mes: Sequence[str], prefixes: Dict[str, Sequence],
                  node_labels: bool = True, adj_labels: bool = True, ucmp: bool = False,
                  binary: bool = True, best_route_selection: bool = False):
        """SpfSolver::buildRouteDb (odl::SpfSolver, C++) for every node in
        `mes`, over SPF results from one batched engine launch.

        prefixes: {prefix: [entry, ...]}, entry = (node, fwd, algo, weight,
        prepend) with fwd 'ip' | 'sr_mpls', algo 'ecmp' | 'ksp2' | 'ucmp_adj'
        | 'ucmp_prefix', weight 0 = unset, prepend None or a label.
        Returns {me: None | {"routes": {prefix: (igp_cost, weight|None)},
        (kind, key): set of (ifName, neighbor, metric, op, labels, weight)}}
        with kind 'U' (prefix) or 'M' (MPLS label) and op 'PHP' | 'SWAP' |
        'PUSH' | 'POP' | ''."""
        lines = _prefix_lines(prefixes)
        flags = int(node_labels) | (2 if adj_labels else 0) | (4 if ucmp else 0) | \
            (8 if best_route_selection else 0)
        if binary and not best_route_selection:  # odl_route_db_bin: records + strings, no text
            return decode_route_db_bin(self.route_db_bin_raw(mes, lines, flags))
        t = self._take(self._L.odl_route_db_text(
            self._h, "\n".join(mes).encode(), len(mes), "\n".join(lines).encode(),
            len(lines), flags))
        return _parse_route_text(t, mes, with_area=False)

    def route_db_bin_raw(self, mes: Sequence[str], prefix_lines: Sequence[str], flags: int) -> bytes:
        """odl_route_db_bin as raw bytes (prefix_lines in the text ABI's
        "prefix\tentries" form): what a C / C++ caller gets, before decoding."""
        buf, nb = C.c_void_p(), C.c_uint64()
        rc = self._L.odl_route_db_bin(self._h, "\n".join(mes).encode(), len(mes),
                                      "\n".join(prefix_lines).encode(), len(prefix_lines), flags,
                                      C.byref(buf), C.byref(nb))
        if rc != 0:
            raise LinkStateError(self._err())
        try:
            return C.string_at(buf.value, nb.value)
        finally:
            self._L.odl_free_buf(buf)

    @staticmethod
    def path_a_in_b(a: Sequence[str], b: Sequence[str]) -> bool:
        """LinkState::pathAInPathB (LinkState.h:477-492) in C++ over link keys."""
        L = N.decision()
        r = L.odl_path_a_in_b("\n".join(a).encode(), len(a), "\n".join(b).encode(), len(b))
        if r < 0:
            raise ValueError(f"malformed link key in {a} / {b}")
        return bool(r)

    def route_db(self, me: str, prefixes: Dict[str, Sequence], **kw):
        """route_dbs for one node."""
        return self.route_dbs([me], prefixes, **kw)[me]

    def ucmp(self, root: str, leaves: Dict[str, int], algo: str = "adj",
             use_link_metric: bool = True):
        """resolveUcmpWeights(getSpfResult(root), leaves, algo) (C++ over the
        GPU SPF result) -> {node: (weight, {iface: (next hop, weight)})}."""
        items = "\n".join(f"{k}\t{v}" for k, v in leaves.items())
        t = self._take(self._L.odl_ucmp_text(self._h, root.encode(), items.encode(),
                                             len(leaves), UCMP_ALGOS[algo],
                                             int(use_link_metric)))
        return parse_ucmp_text(t)

    def links(self, node: str):
        out = []
        for ln in self._take(self._L.odl_links_text(self._h, node.encode())).splitlines():
            key, m, up = ln.split("\t")
            out.append((key, int(m), up == "1"))
        return out

    linksFromNode = links

    def link_keys(self) -> List[str]:
        """Link keys of the current snapshot in link id order (ids of csr()
        and of the engine's KSP2 records)."""
        return self._take(self._L.odl_link_keys_text(self._h)).splitlines()

    def metric(self, a: str, b: str, use_link_metric: bool = True) -> Optional[int]:
        v = self._L.odl_metric_a_to_b(self._h, a.encode(), b.encode(), int(use_link_metric))
        if v == -2:
            raise LinkStateError(self._err())
        return None if v < 0 else v

    getMetricFromAToB = metric

    def is_overloaded(self, node: str) -> bool:
        return bool(self._L.odl_is_overloaded(self._h, node.encode()))

    isNodeOverloaded = is_overloaded

    @property
    def spf_runs(self) -> int:
        return int(self._L.odl_spf_runs(self._h))

    def set_incremental(self, on: bool = True) -> None:
        """Keep memoised SPF results a metric / up / overload-only update
        cannot affect (odl_set_incremental; off = the reference's behaviour)."""
        self._L.odl_set_incremental(self._h, int(on))

    def apply_kvs(self, key_vals, expired=(), my_node: Optional[str] = None):
        """Decision::processPublication's LinkState part (odl_apply_kvs):
        key_vals = [(key, compact-thrift AdjacencyDatabase bytes or None)] in
        keyVals iteration order, then expired keys. Change records as tuples
        (topology, link attributes, node label, added links)."""
        n, ne = len(key_vals), len(expired)
        keys = (C.c_char_p * max(n, 1))(*[k.encode() for k, _ in key_vals])
        bufs = [v for _, v in key_vals]
        vals = (C.c_void_p * max(n, 1))(*[(C.cast(C.c_char_p(v), C.c_void_p).value if v is not None
                                            else None) for v in bufs])
        lens = (C.c_uint64 * max(n, 1))(*[len(v) if v is not None else 0 for v in bufs])
        exp = (C.c_char_p * max(ne, 1))(*[k.encode() for k in expired])
        ch = change_array(n + ne)
        if self._L.odl_apply_kvs(self._h, n, keys, vals, lens, ne, exp,
                                 my_node.encode() if my_node is not None else None, ch) != 0:
            raise LinkStateError(self._err())
        self.decode_errors = [i for i in range(n + ne) if ch[i].decode_error]
        return changes_to_list(ch, n + ne)

    def apply_publication(self, buf: bytes, my_node: Optional[str] = None):
        """A whole compact-thrift thrift::Publication (odl_apply_publication).
        Values that fail to decode skip their own key only: their record
        indices are left in self.decode_errors, the reason in
        last_decode_error()."""
        nout = C.c_uint32(0)
        cap = 64
        me = my_node.encode() if my_node is not None else None
        while True:
            ch = change_array(cap)
            rc = self._L.odl_apply_publication(self._h, buf, len(buf), me, ch, cap, C.byref(nout))
            if rc == -2 and int(nout.value) > cap:  # ODL_E_SMALL: nothing applied
                cap = int(nout.value)
                continue
            if rc != 0:
                raise LinkStateError(self._err())
            break
        n = int(nout.value)
        self.decode_errors = [i for i in range(n) if ch[i].decode_error]
        return changes_to_list(ch, n)

    def counters(self) -> dict:
        """The path's fb303 counters (odl_get_counters): decision.spf_runs,
        spf_ms / ucmp_ms / route_build_ms as sums + sample counts (AVG =
        sum / samples), ucmp_runs, and the device errors survived."""
        c = N.odl_counters()
        self._L.odl_get_counters(self._h, C.byref(c))
        return {k: getattr(c, k) for k, _ in c._fields_}

    def set_degrade(self, on: bool = True) -> None:
        """Degrade to the host path on device errors (odl_set_degrade)."""
        self._L.odl_set_degrade(self._h, int(on))

    def last_engine_error(self) -> str:
        return (self._L.odl_last_engine_error(self._h) or b"").decode()

    def inject_engine_error(self, after: int = 1) -> None:
        """Test hook: the after-th engine call from now fails (OSPF_E_DEVICE)."""
        if self._L.odl_inject_engine_error(self._h, after) != 0:
            raise LinkStateError(self._err())

    def last_decode_error(self):
        """(message of the last value that failed to decode or "", count so far)."""
        k = C.c_uint64(0)
        msg = self._L.odl_last_decode_error(self._h, C.byref(k))
        return (msg or b"").decode(), int(k.value)

    def set_host_spf(self, on: bool = True) -> None:
        """Run every SPF / KSP2 / digest of this LinkState on the host with the
        reference's algorithm, the engine never opened (odl_set_host_spf): a
        GPU-free run of the ingest / patch / memo logic, for sanitizer builds
        and CPU tests. Off by default."""
        self._L.odl_set_host_spf(self._h, int(on))

    def incremental_stats(self) -> Dict[str, int]:
        out = (C.c_uint64 * 3)()
        self._L.odl_incremental_stats(self._h, out)
        return {"patches": int(out[0]), "kept": int(out[1]), "dropped": int(out[2])}

    @property
    def node_patches(self) -> int:
        """nodes added / removed in place (odl_node_patches)"""
        return int(self._L.odl_node_patches(self._h))

    def shard_stats(self) -> Dict[str, int]:
        """multi-device LinkState: root batches / KSP2 prefetches split across
        the device slots and their per-slot launches (odl_shard_stats)"""
        out = (C.c_uint64 * 4)()
        self._L.odl_shard_stats(self._h, out)
        return {"spf_batches": int(out[0]), "spf_launches": int(out[1]),
                "ksp2_runs": int(out[2]), "ksp2_launches": int(out[3])}

    def topology_stats(self) -> Dict[str, int]:
        """{snapshots, loads, link_patches, rows_patched}: links added /
        removed between known nodes patch the CSR and the device graph in
        place (odl_topology_stats)."""
        out = (C.c_uint64 * 4)()
        self._L.odl_topology_stats(self._h, out)
        return {"snapshots": int(out[0]), "loads": int(out[1]), "link_patches": int(out[2]),
                "rows_patched": int(out[3])}

    def num_nodes(self) -> int:
        return int(self._L.odl_num_nodes(self._h))

    def num_links(self) -> int:
        return int(self._L.odl_num_links(self._h))

    # ------------------------------------------------------------ batches
    def digests(self, roots: Sequence[str], use_link_metric: bool = True) -> np.ndarray:
        out = np.zeros((len(roots), 3), np.uint64)
        if self._L.odl_spf_digests(self._h, "\n".join(roots).encode(), len(roots),
                                   int(use_link_metric), out.ctypes.data) != 0:
            raise LinkStateError(self._err())
        return out

    def all_sources_digests(self, use_link_metric: bool = True) -> np.ndarray:
        """Digests of every node (node id order) from one all-sources sweep."""
        out = np.zeros((self.num_nodes(), 3), np.uint64)
        if self._L.odl_all_sources_digests(self._h, int(use_link_metric), out.ctypes.data) != 0:
            raise LinkStateError(self._err())
        return out

    def prefetch_all(self, use_link_metric: bool = True) -> None:
        if self._L.odl_all_sources_prefetch(self._h, int(use_link_metric)) != 0:
            raise LinkStateError(self._err())

    def sweep_stats(self) -> Dict[str, int]:
        out = (C.c_uint64 * 5)()
        self._L.odl_sweep_stats(self._h, out)
        return {"sweeps": int(out[0]), "rows_copied": int(out[1]),
                "mode": N.SWEEP_MODE_NAMES.get(int(out[2]), str(out[2])),
                "devices": int(out[3]), "hip_graph": int(out[4])}

    def prefetch(self, roots: Sequence[str], use_link_metric: bool = True) -> None:
        if self._L.odl_spf_prefetch(self._h, "\n".join(roots).encode(), len(roots),
                                    int(use_link_metric)) != 0:
            raise LinkStateError(self._err())

    # ------------------------------------------------------------ snapshot
    def csr(self) -> Dict[str, np.ndarray]:
        V, E = C.c_uint32(), C.c_uint32()
        if self._L.odl_csr_size(self._h, C.byref(V), C.byref(E)) != 0:
            raise LinkStateError(self._err())
        V, E = V.value, E.value
        a = dict(row_ptr=np.zeros(V + 1, np.uint32), col=np.zeros(E, np.uint32),
                 metric=np.zeros(E, np.uint32), link_id=np.zeros(E, np.uint32),
                 twin=np.zeros(E, np.uint32), edge_up=np.zeros(E, np.uint8),
                 no_transit=np.zeros(V, np.uint8), link_rank=np.zeros(E, np.uint32))
        ptrs = [a[k].ctypes.data if a[k].size else None for k in
                ("row_ptr", "col", "metric", "link_id", "twin", "edge_up", "no_transit",
                 "link_rank")]
        if self._L.odl_csr_export(self._h, *ptrs) != 0:
            raise LinkStateError(self._err())
        return a

    def node_names(self) -> List[str]:
        n = self.num_nodes()
        return [self._L.odl_node_name(self._h, i).decode() for i in range(n)]

    def node_id(self, name: str) -> int:
        return int(self._L.odl_node_id(self._h, name.encode()))
