"""Compact-protocol thrift ENCODER for the test side (test infrastructure):
builds the bytes KvStore would carry -- thrift::AdjacencyDatabase /
Adjacency (openr/if/Types.thrift:98-207), thrift::Value and
thrift::Publication (openr/if/KvStore.thrift:177-225, 270-320) -- from the
published Apache Thrift compact protocol (TCompactProtocol), so the product's
decoder (openr_amd/csrc/decision/adjdb_thrift.cpp) is checked against an
independent writer. fbthrift / folly are not in this image, so the bytes are
not cross-checked against fbthrift's own serializer; the known-answer vectors
in tests/test_host_publication.py are worked out by hand from the protocol.
Fields are written in the IDL's declaration order (as fbthrift's generated
code writes them), which exercises out-of-order ids (Adjacency: 1, 2, 3, 5,
4, 6, ...) and the long field-header form."""
from __future__ import annotations

import struct as _st
from typing import Iterable, List, Optional, Sequence, Tuple

T_TRUE, T_FALSE, T_BYTE, T_I16, T_I32, T_I64, T_DOUBLE, T_BINARY, T_LIST, T_SET, T_MAP, T_STRUCT = \
    1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12


def varint(n: int) -> bytes:
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def zigzag(n: int, bits: int = 64) -> int:
    return (n << 1) ^ (n >> (bits - 1))


class Writer:
    def __init__(self):
        self.buf = bytearray()
        self.last = [0]

    def field(self, fid: int, ftype: int):
        d = fid - self.last[-1]
        if 0 < d <= 15:
            self.buf.append((d << 4) | ftype)
        else:
            self.buf.append(ftype)
            self.buf += varint(zigzag(fid, 16) & 0xFFFF)
        self.last[-1] = fid

    def begin(self):
        self.last.append(0)

    def end(self):
        self.buf.append(0)
        self.last.pop()

    def string(self, fid: int, s):
        b = s.encode() if isinstance(s, str) else bytes(s)
        self.field(fid, T_BINARY)
        self.buf += varint(len(b)) + b

    def i32(self, fid: int, v: int):
        self.field(fid, T_I32)
        self.buf += varint(zigzag(v, 32) & 0xFFFFFFFF)

    def i64(self, fid: int, v: int):
        self.field(fid, T_I64)
        self.buf += varint(zigzag(v, 64) & 0xFFFFFFFFFFFFFFFF)

    def boolean(self, fid: int, v: bool):
        self.field(fid, T_TRUE if v else T_FALSE)

    def list_header(self, fid: int, etype: int, n: int):
        self.field(fid, T_LIST)
        if n < 15:
            self.buf.append((n << 4) | etype)
        else:
            self.buf.append(0xF0 | etype)
            self.buf += varint(n)

    def binary_address(self, fid: int, addr: bytes, if_name: Optional[str] = None):
        """Network.BinaryAddress {1: binary addr, 3: optional string ifName}"""
        self.field(fid, T_STRUCT)
        self.begin()
        self.string(1, addr)
        if if_name is not None:
            self.string(3, if_name)
        self.end()


def write_adjacency(w: Writer, a, extra: bool = True):
    """a: openr_amd.adjdb.Adjacency; IDL order 1, 2, 3, 5, 4, 6 .. 12"""
    w.begin()
    w.string(1, a.other)
    w.string(2, a.if_name)
    if extra:
        w.binary_address(3, bytes([0xFE, 0x80] + [0] * 13 + [1]))
        w.binary_address(5, bytes([10, 0, 0, 1]))
    w.i32(4, a.metric)
    w.i32(6, a.label)
    w.boolean(7, a.overloaded)
    if extra:
        w.i32(8, 1234)        # rtt
        w.i64(9, 1700000000)  # timestamp
    w.i64(10, a.weight)
    w.string(11, a.other_if)
    w.boolean(12, a.only_used_by_other)
    w.end()


def adjacency_database(db, area: str = "0", perf: bool = True, extra: bool = True) -> bytes:
    """CompactSerializer bytes of thrift::AdjacencyDatabase for an
    openr_amd.adjdb.AdjDb (with perfEvents and area, as Decision receives them)."""
    w = Writer()
    w.begin()
    w.string(1, db.name)
    w.boolean(2, db.overloaded)
    w.list_header(3, T_STRUCT, len(db.adjs))
    for a in db.adjs:
        write_adjacency(w, a, extra)
    w.i32(4, db.node_label)
    if perf:  # 5: optional PerfEvents {1: list<PerfEvent{1 nodeName, 2 eventDescr, 3 unixTs}>}
        w.field(5, T_STRUCT)
        w.begin()
        w.list_header(1, T_STRUCT, 1)
        w.begin()
        w.string(1, db.name)
        w.string(2, "DECISION_INIT_UPDATE")
        w.i64(3, 1700000000123)
        w.end()
        w.end()
    w.string(6, area)
    w.end()
    return bytes(w.buf)


def value(data: Optional[bytes], version: int = 1, originator: str = "node", ttl: int = 3600000,
          ttl_version: int = 0) -> bytes:
    """thrift::Value bytes (1 version, 3 originatorId, 2 optional value, 4 ttl,
    5 ttlVersion): IDL order; data None = a TTL-only update."""
    w = Writer()
    w.begin()
    w.i64(1, version)
    w.string(3, originator)
    if data is not None:
        w.string(2, data)
    w.i64(4, ttl)
    w.i64(5, ttl_version)
    w.end()
    return bytes(w.buf)


def publication(key_vals: Sequence[Tuple[str, bytes]], expired: Sequence[str] = (),
                area: str = "0", node_ids: Sequence[str] = ("n1",)) -> bytes:
    """thrift::Publication bytes: 2 keyVals map<string, Value> (wire order =
    the given order), 3 expiredKeys, 4 nodeIds, 7 area. key_vals values are
    encoded thrift::Value structs (value())."""
    w = Writer()
    w.begin()
    w.field(2, T_MAP)
    w.buf += varint(len(key_vals))
    if key_vals:
        w.buf.append((T_BINARY << 4) | T_STRUCT)
        for k, v in key_vals:
            kb = k.encode()
            w.buf += varint(len(kb)) + kb
            w.buf += v  # a whole struct (ends with its stop byte)
    w.list_header(3, T_BINARY, len(expired))
    for k in expired:
        kb = k.encode()
        w.buf += varint(len(kb)) + kb
    w.list_header(4, T_BINARY, len(node_ids))
    for k in node_ids:
        kb = k.encode()
        w.buf += varint(len(kb)) + kb
    w.string(7, area)
    w.end()
    return bytes(w.buf)
