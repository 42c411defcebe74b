"""Columnar AdjacencyDatabase update streams (``include/openr_adjdb.h``).

An :class:`AdjDbStream` is an ordered list of ``LinkState::updateAdjacencyDatabase``
/ ``deleteAdjacencyDatabase`` calls (openr/decision/LinkState.cpp:584,730) with the
thrift fields LinkState reads (openr/if/Types.thrift:98-207). It is frozen into
numpy columns and handed to the C libraries as an ``oadj_stream`` struct.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional, Sequence

import numpy as np


@dataclass
class Adjacency:
    """thrift::Adjacency (Types.thrift:98-168), SPF-relevant fields only."""

    other: str
    if_name: str
    other_if: str
    metric: int = 1
    label: int = 0
    overloaded: bool = False
    weight: int = 1
    only_used_by_other: bool = False


@dataclass
class AdjDb:
    """thrift::AdjacencyDatabase (Types.thrift:175-207)."""

    name: str
    adjs: List[Adjacency] = field(default_factory=list)
    node_label: int = 0
    overloaded: bool = False
    delete: bool = False


def create_adjacency(node: str, if_name: str, remote_if: str, metric: int = 1,
                     label: int = 0, weight: int = 1, only_used_by_other: bool = False,
                     overloaded: bool = False) -> Adjacency:
    """Mirror of openr::createAdjacency (openr/common/LsdbUtil.cpp:462-485)."""
    return Adjacency(node, if_name, remote_if, metric, label, overloaded, weight,
                     only_used_by_other)


class oadj_stream(C.Structure):  # noqa: N801 - C name
    _fields_ = [
        ("str_data", C.c_void_p),
        ("str_off", C.c_void_p),
        ("n_str", C.c_uint32),
        ("n_dbs", C.c_uint32),
        ("db_name", C.c_void_p),
        ("db_overloaded", C.c_void_p),
        ("db_node_label", C.c_void_p),
        ("db_delete", C.c_void_p),
        ("db_adj_off", C.c_void_p),
        ("adj_other", C.c_void_p),
        ("adj_if", C.c_void_p),
        ("adj_other_if", C.c_void_p),
        ("adj_metric", C.c_void_p),
        ("adj_label", C.c_void_p),
        ("adj_overloaded", C.c_void_p),
        ("adj_weight", C.c_void_p),
        ("adj_only_used_by_other", C.c_void_p),
    ]


class oadj_change(C.Structure):  # noqa: N801
    _fields_ = [
        ("topology_changed", C.c_int32),
        ("link_attributes_changed", C.c_int32),
        ("node_label_changed", C.c_int32),
        ("n_added_links", C.c_int32),
        ("decode_error", C.c_int32),
    ]


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data if a.size else 0


class AdjDbStream:
    """Frozen columnar stream. Keep the object alive while a C call reads it."""

    def __init__(self, strings: Sequence[str], cols: Dict[str, np.ndarray]):
        self.strings = list(strings)
        enc = [s.encode() for s in self.strings]
        lens = np.fromiter((len(b) for b in enc), dtype=np.uint64, count=len(enc))
        self.str_off = np.zeros(len(enc) + 1, dtype=np.uint64)
        np.cumsum(lens, out=self.str_off[1:])
        self.str_data = np.frombuffer(b"".join(enc) or b"\0", dtype=np.uint8).copy()
        self.cols = {k: np.ascontiguousarray(v) for k, v in cols.items()}
        c = self.cols
        self.n_dbs = int(c["db_name"].size)
        self.struct = oadj_stream(
            _ptr(self.str_data), _ptr(self.str_off), len(enc), self.n_dbs,
            _ptr(c["db_name"]), _ptr(c["db_overloaded"]), _ptr(c["db_node_label"]),
            _ptr(c["db_delete"]), _ptr(c["db_adj_off"]), _ptr(c["adj_other"]),
            _ptr(c["adj_if"]), _ptr(c["adj_other_if"]), _ptr(c["adj_metric"]),
            _ptr(c["adj_label"]), _ptr(c["adj_overloaded"]), _ptr(c["adj_weight"]),
            _ptr(c["adj_only_used_by_other"]))

    @property
    def n_adjs(self) -> int:
        return int(self.cols["adj_other"].size)

    def ref(self) -> C.POINTER(oadj_stream):
        return C.pointer(self.struct)

    def db_names(self) -> List[str]:
        return [self.strings[i] for i in self.cols["db_name"]]

    @staticmethod
    def from_dbs(dbs: Iterable[AdjDb]) -> "AdjDbStream":
        table: Dict[str, int] = {}
        strings: List[str] = []

        def sid(s: str) -> int:
            i = table.get(s)
            if i is None:
                i = table[s] = len(strings)
                strings.append(s)
            return i

        db_name, db_ov, db_lbl, db_del, db_off = [], [], [], [], [0]
        a_other, a_if, a_oif, a_met, a_lbl, a_ov, a_w, a_only = ([] for _ in range(8))
        for db in dbs:
            db_name.append(sid(db.name))
            db_ov.append(int(db.overloaded))
            db_lbl.append(db.node_label)
            db_del.append(int(db.delete))
            for a in db.adjs:
                a_other.append(sid(a.other))
                a_if.append(sid(a.if_name))
                a_oif.append(sid(a.other_if))
                a_met.append(a.metric)
                a_lbl.append(a.label)
                a_ov.append(int(a.overloaded))
                a_w.append(a.weight)
                a_only.append(int(a.only_used_by_other))
            db_off.append(len(a_other))
        cols = dict(
            db_name=np.array(db_name, np.uint32), db_overloaded=np.array(db_ov, np.uint8),
            db_node_label=np.array(db_lbl, np.int32), db_delete=np.array(db_del, np.uint8),
            db_adj_off=np.array(db_off, np.uint64), adj_other=np.array(a_other, np.uint32),
            adj_if=np.array(a_if, np.uint32), adj_other_if=np.array(a_oif, np.uint32),
            adj_metric=np.array(a_met, np.int32), adj_label=np.array(a_lbl, np.int32),
            adj_overloaded=np.array(a_ov, np.uint8), adj_weight=np.array(a_w, np.int64),
            adj_only_used_by_other=np.array(a_only, np.uint8))
        return AdjDbStream(strings, cols)

    def to_dbs(self) -> List[AdjDb]:
        c, s = self.cols, self.strings
        out = []
        for i in range(self.n_dbs):
            lo, hi = int(c["db_adj_off"][i]), int(c["db_adj_off"][i + 1])
            adjs = [Adjacency(s[c["adj_other"][a]], s[c["adj_if"][a]], s[c["adj_other_if"][a]],
                              int(c["adj_metric"][a]), int(c["adj_label"][a]),
                              bool(c["adj_overloaded"][a]), int(c["adj_weight"][a]),
                              bool(c["adj_only_used_by_other"][a])) for a in range(lo, hi)]
            out.append(AdjDb(s[c["db_name"][i]], adjs, int(c["db_node_label"][i]),
                             bool(c["db_overloaded"][i]), bool(c["db_delete"][i])))
        return out


def change_array(n: int):
    return (oadj_change * max(n, 1))()


def changes_to_list(arr, n: int) -> List[tuple]:
    return [(bool(arr[i].topology_changed), bool(arr[i].link_attributes_changed),
             bool(arr[i].node_label_changed), int(arr[i].n_added_links)) for i in range(n)]


def merge(*streams: Optional[AdjDbStream]) -> AdjDbStream:
    dbs: List[AdjDb] = []
    for s in streams:
        if s is not None:
            dbs.extend(s.to_dbs())
    return AdjDbStream.from_dbs(dbs)


def decode_adjdbs(values: Sequence[bytes]) -> AdjDbStream:
    """Compact-thrift thrift::AdjacencyDatabase values (KvStore "adj:" keys)
    decoded on host threads by libopenr_decision (odl_adjdbs_decode) into a
    columnar stream; the columns are copied out and the C object freed."""
    from . import _native as N
    L = N.decision()
    n = len(values)
    keep = [bytes(v) for v in values]
    ptrs = (C.c_void_p * max(n, 1))(*[C.cast(C.c_char_p(v), C.c_void_p).value for v in keep])
    lens = (C.c_uint64 * max(n, 1))(*[len(v) for v in keep])
    h = L.odl_adjdbs_decode(ptrs, lens, n)
    if not h:
        raise ValueError("odl_adjdbs_decode: " + L.odl_adjdbs_error().decode())
    try:
        s = oadj_stream.from_address(L.odl_adjdbs_stream(h))

        def col(ptr, count, dt):
            if count == 0:
                return np.zeros(0, dt)
            return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(np.ctypeslib.as_ctypes_type(dt))),
                                         (count,)).copy()
        n_dbs, n_str = s.n_dbs, s.n_str
        adj_off = col(s.db_adj_off, n_dbs + 1, np.uint64)
        na = int(adj_off[-1]) if n_dbs else 0
        str_off = col(s.str_off, n_str + 1, np.uint64)
        data = C.string_at(s.str_data, int(str_off[-1])) if n_str else b""
        strings = [data[int(str_off[i]):int(str_off[i + 1])].decode() for i in range(n_str)]
        cols = dict(
            db_name=col(s.db_name, n_dbs, np.uint32), db_overloaded=col(s.db_overloaded, n_dbs, np.uint8),
            db_node_label=col(s.db_node_label, n_dbs, np.int32), db_delete=col(s.db_delete, n_dbs, np.uint8),
            db_adj_off=adj_off, adj_other=col(s.adj_other, na, np.uint32),
            adj_if=col(s.adj_if, na, np.uint32), adj_other_if=col(s.adj_other_if, na, np.uint32),
            adj_metric=col(s.adj_metric, na, np.int32), adj_label=col(s.adj_label, na, np.int32),
            adj_overloaded=col(s.adj_overloaded, na, np.uint8), adj_weight=col(s.adj_weight, na, np.int64),
            adj_only_used_by_other=col(s.adj_only_used_by_other, na, np.uint8))
        if n_dbs == 0:
            cols["db_adj_off"] = np.zeros(1, np.uint64)
        return AdjDbStream(strings, cols)
    finally:
        L.odl_adjdbs_free(h)
