"""The binary route-DB records (odl_route_db_bin, include/openr_decision.h):
the numpy reader decodes a hand-built buffer into route_dbs' dict -- the same
shape the text ABI gives (the GPU test compares the two on real builds)."""
import numpy as np

from openr_amd import _native as N
from openr_amd.linkstate import (RDB_HEADER, RDB_MAGIC, RDB_NH, RDB_NODE, RDB_ROUTE,
                                 decode_route_db_bin)


def build(nodes, routes, nhs, labels, strs):
    def al(x):
        return (x + 7) & ~7
    hd = np.zeros(1, RDB_HEADER)
    off_nodes = al(RDB_HEADER.itemsize)
    off_routes = al(off_nodes + RDB_NODE.itemsize * len(nodes))
    off_nhs = al(off_routes + RDB_ROUTE.itemsize * len(routes))
    off_labels = al(off_nhs + RDB_NH.itemsize * len(nhs))
    off_strings = al(off_labels + 4 * len(labels))
    total = al(off_strings + len(strs))
    hd[0] = (RDB_MAGIC, 1, total, len(nodes), len(routes), len(nhs), len(labels), off_nodes,
             off_routes, off_nhs, off_labels, off_strings, len(strs))
    buf = bytearray(total)
    buf[0:RDB_HEADER.itemsize] = hd.tobytes()
    buf[off_nodes:off_nodes + RDB_NODE.itemsize * len(nodes)] = np.array(nodes, RDB_NODE).tobytes()
    buf[off_routes:off_routes + RDB_ROUTE.itemsize * len(routes)] = np.array(routes, RDB_ROUTE).tobytes()
    buf[off_nhs:off_nhs + RDB_NH.itemsize * len(nhs)] = np.array(nhs, RDB_NH).tobytes()
    buf[off_labels:off_labels + 4 * len(labels)] = np.array(labels, "<i4").tobytes()
    buf[off_strings:off_strings + len(strs)] = strs
    return bytes(buf)


def test_decode_route_db_bin():
    strs = b"me1\x00me2\x0010.0.0.0/24\x00if-a\x00nbr-a\x00if-b\x00nbr-b\x00"
    o = {}
    pos = 0
    for x in strs.split(b"\x00")[:-1]:
        o[x.decode()] = pos
        pos += len(x) + 1
    nodes = [(o["me1"], 1, 0, 1, 1, 0), (o["me2"], 0, 2, 0, 0, 0)]
    routes = [(0, o["10.0.0.0/24"], 20, 1, 5, 0, 2),          # unicast, 2 next hops
              (1, 0xFFFFFFFF & 100010, 0, 0, 0, 2, 1)]         # MPLS label 100010
    nhs = [(o["if-a"], o["nbr-a"], 10, 0, 0, 0, 0, 0),
           (o["if-b"], o["nbr-b"], 20, 3, 3, 0, 2, 0),         # PUSH 2 labels
           (o["if-a"], o["nbr-a"], 10, 0, 2, 2, 1, 0)]         # SWAP 1 label
    labels = [7, 8, 100011]
    got = decode_route_db_bin(build(nodes, routes, nhs, labels, strs))
    assert got["me2"] is None
    db = got["me1"]
    assert db["routes"] == {"10.0.0.0/24": (20, 5)}
    assert db[("U", "10.0.0.0/24")] == {("if-a", "nbr-a", 10, "", (), 0),
                                        ("if-b", "nbr-b", 20, "PUSH", (7, 8), 3)}
    assert db[("M", "100010")] == {("if-a", "nbr-a", 10, "SWAP", (100011,), 0)}


def test_route_db_bin_symbols_exported():
    L = N.decision()
    assert hasattr(L, "odl_route_db_bin") and hasattr(L, "odl_free_buf")
