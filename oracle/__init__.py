"""CPU oracle for the OpenR SPF hot path — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this package, and only as the checker / timed CPU baseline. The product
package (openr_amd) never imports it.

Python face of oracle/linkstate_oracle.cpp (see its header for the reference
file:line each piece restates).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from typing import List, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.environ.get("OPENR_ORACLE_SO") or os.path.join(_HERE, "build", "liboracle.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _SO


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = C.CDLL(_SO)
        vp, cp, u32, i32, u64 = C.c_void_p, C.c_char_p, C.c_uint32, C.c_int, C.c_uint64
        L.orc_create.restype = vp
        L.orc_destroy.argtypes = [vp]
        L.orc_free.argtypes = [vp]
        L.orc_apply.argtypes = [vp, vp, u32, u32, vp]
        for f in ("orc_spf_text", "orc_kth_paths_text", "orc_links_text", "orc_ksp2_text",
                  "orc_ucmp_text", "orc_ksp2_text_threads"):
            getattr(L, f).restype = C.POINTER(C.c_char)
        L.orc_spf_text.argtypes = [vp, cp, i32]
        L.orc_kth_paths_text.argtypes = [vp, cp, cp, i32]
        L.orc_links_text.argtypes = [vp, cp]
        L.orc_ksp2_text.argtypes = [vp, cp, cp, u32]
        L.orc_ksp2_text_threads.argtypes = [vp, cp, cp, u32, i32]
        L.orc_ucmp_text.argtypes = [vp, cp, cp, u32, i32, i32]
        L.orc_metric_a_to_b.argtypes = [vp, cp, cp, i32]
        L.orc_metric_a_to_b.restype = C.c_int64
        L.orc_spf_runs.argtypes = [vp]
        L.orc_spf_runs.restype = u64
        L.orc_num_nodes.argtypes = [vp]
        L.orc_num_nodes.restype = u32
        L.orc_num_links.argtypes = [vp]
        L.orc_num_links.restype = u32
        L.orc_is_overloaded.argtypes = [vp, cp]
        L.orc_digest_roots.argtypes = [vp, cp, u32, i32, i32, vp]
        L.orc_fast_digest_roots.argtypes = [vp, cp, u32, i32, i32, vp]
        L.orc_intmap_order.argtypes = [vp, u32, vp]
        _lib = L
    return _lib


def _take(p) -> str:
    s = C.cast(p, C.c_char_p).value.decode()
    lib().orc_free(p)
    return s


def intmap_order(keys: Sequence[int]) -> List[int]:
    k = np.asarray(keys, np.int32)
    out = np.zeros(len(k), np.int32)
    n = lib().orc_intmap_order(k.ctypes.data, len(k), out.ctypes.data)
    return out[:n].tolist()


class Oracle:
    """Reference-shaped LinkState (CPU)."""

    def __init__(self, stream=None):
        self._h = lib().orc_create()
        if stream is not None:
            self.apply(stream)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().orc_destroy(self._h)
            self._h = None

    def apply(self, stream, first: int = 0, count: int = None):
        from openr_amd.adjdb import change_array, changes_to_list  # data format only
        count = stream.n_dbs - first if count is None else count
        ch = change_array(count)
        rc = lib().orc_apply(self._h, C.addressof(stream.struct), first, count, C.addressof(ch))
        if rc:
            raise RuntimeError("orc_apply failed")
        return changes_to_list(ch, count)

    def spf_text(self, root: str, use_link_metric: bool = True) -> str:
        return _take(lib().orc_spf_text(self._h, root.encode(), int(use_link_metric)))

    def kth_paths(self, src: str, dst: str, k: int) -> List[List[str]]:
        t = _take(lib().orc_kth_paths_text(self._h, src.encode(), dst.encode(), k))
        return [ln.split(",") for ln in t.splitlines()]

    def ksp2_text(self, src: str, dsts: Sequence[str], threads: int = 1) -> str:
        if threads > 1:
            return _take(lib().orc_ksp2_text_threads(self._h, src.encode(),
                                                     "\n".join(dsts).encode(), len(dsts),
                                                     threads))
        return _take(lib().orc_ksp2_text(self._h, src.encode(),
                                         "\n".join(dsts).encode(), len(dsts)))

    def ucmp(self, root: str, leaves, algo: str = "adj", use_link_metric: bool = True):
        """resolveUcmpWeights restated -> {node: (weight, {iface: (next hop, weight)})}."""
        from openr_amd.linkstate import UCMP_ALGOS, parse_ucmp_text  # text format only
        items = "\n".join(f"{k}\t{v}" for k, v in leaves.items())
        return parse_ucmp_text(_take(lib().orc_ucmp_text(
            self._h, root.encode(), items.encode(), len(leaves), UCMP_ALGOS[algo],
            int(use_link_metric))))

    def links_text(self, node: str) -> str:
        return _take(lib().orc_links_text(self._h, node.encode()))

    def metric(self, a: str, b: str, use_link_metric: bool = True):
        v = lib().orc_metric_a_to_b(self._h, a.encode(), b.encode(), int(use_link_metric))
        return None if v < 0 else v

    @property
    def spf_runs(self) -> int:
        return lib().orc_spf_runs(self._h)

    def num_nodes(self) -> int:
        return lib().orc_num_nodes(self._h)

    def num_links(self) -> int:
        return lib().orc_num_links(self._h)

    def is_overloaded(self, n: str) -> bool:
        return bool(lib().orc_is_overloaded(self._h, n.encode()))

    def digests(self, roots: Sequence[str], use_link_metric: bool = True,
                threads: int = 1) -> np.ndarray:
        """Un-memoized runSpf per root -> (n,3) u64 {reached, sumDist, digest}."""
        out = np.zeros((len(roots), 3), np.uint64)
        lib().orc_digest_roots(self._h, "\n".join(roots).encode(), len(roots),
                               int(use_link_metric), threads, out.ctypes.data)
        return out

    def fast_digests(self, roots: Sequence[str], use_link_metric: bool = True,
                     threads: int = 1) -> np.ndarray:
        """Same digests from the CSR-Dijkstra restatement (integer ids, binary
        heap): the checker for weighted graphs at scale, where the
        reference-shaped heap's make_heap per improvement is quadratic."""
        out = np.zeros((len(roots), 3), np.uint64)
        lib().orc_fast_digest_roots(self._h, "\n".join(roots).encode(), len(roots),
                                    int(use_link_metric), threads, out.ctypes.data)
        return out


def parse_spf_text(t: str):
    """-> {name: (metric, tuple(nexthops), tuple(pathlinks))}"""
    out = {}
    for ln in t.splitlines():
        name, metric, nh, pl = ln.split("\t")
        out[name] = (int(metric), tuple(x for x in nh.split(",") if x),
                     tuple(x for x in pl.split(";") if x))
    return out
