"""Python face of libopenr_spf_hip (include/openr_spf.h).

``Engine`` owns one ospf_ctx on a HIP device. ``run`` is the synchronous
host-buffer batch (the drop-in ``ospf_sssp_batch``); ``run_dev`` queues a
device-resident batch on a stream (raw device pointers, e.g. from torch
tensors' ``data_ptr()``) — that is what bench.py times.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, Optional, Sequence

import numpy as np

from . import _native as N


class EngineError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"ospf error {code}: {msg}")
        self.code = code


def csr_struct(csr: Dict[str, np.ndarray]):
    keep = {k: np.ascontiguousarray(v) for k, v in csr.items()}
    s = N.ospf_csr(int(keep["row_ptr"].size - 1), int(keep["col"].size),
                   keep["row_ptr"].ctypes.data, keep["col"].ctypes.data,
                   keep["metric"].ctypes.data, keep["link_id"].ctypes.data,
                   keep["twin"].ctypes.data, keep["edge_up"].ctypes.data,
                   keep["no_transit"].ctypes.data,
                   keep["link_rank"].ctypes.data if "link_rank" in keep else None)
    return s, keep


def decode_paths(recs: np.ndarray, status: np.ndarray, bad: int):
    """KSP2 records -> per row a list of paths (lists of link ids), None when
    `status & bad`."""
    out = []
    for rec, st in zip(recs, status):
        if int(st) & bad:
            out.append(None)
            continue
        paths, q = [], 1
        for _ in range(int(rec[0])):
            ln = int(rec[q])
            paths.append([int(x) for x in rec[q + 1:q + 1 + ln]])
            q += 1 + ln
        out.append(paths)
    return out


class Engine:
    def __init__(self, device: int = 0):
        self._L = N.engine()
        h = C.c_void_p()
        rc = self._L.ospf_open(device, C.byref(h))
        if rc != 0:
            raise EngineError(rc, f"ospf_open(device={device}) failed: no usable HIP device")
        self._h = h
        self.V = 0

    def close(self):
        if getattr(self, "_h", None):
            self._L.ospf_close(self._h)
            self._h = None

    __del__ = close

    def _check(self, rc: int):
        if rc != 0:
            raise EngineError(rc, self._L.ospf_last_error(self._h).decode())

    def load(self, csr: Dict[str, np.ndarray], version: int = 1) -> None:
        s, keep = csr_struct(csr)
        self._check(self._L.ospf_load_graph(self._h, C.byref(s), version))
        self.V = int(s.n_nodes)

    def info(self) -> N.ospf_graph_info:
        gi = N.ospf_graph_info()
        self._check(self._L.ospf_graph_info_get(self._h, C.byref(gi)))
        return gi

    def root_neighbors(self, root: int) -> np.ndarray:
        n = C.c_uint32()
        self._check(self._L.ospf_root_neighbors(self._h, root, None, 0, C.byref(n)))
        ids = np.zeros(max(n.value, 1), np.uint32)
        self._check(self._L.ospf_root_neighbors(self._h, root, ids.ctypes.data, n.value,
                                                C.byref(n)))
        return ids[: n.value]

    def nh_words(self, root: int) -> int:
        return max(1, (len(self.root_neighbors(root)) + 31) // 32)

    def plan_variant(self, nh_words: int, flags: int = 0) -> int:
        v = C.c_int()
        self._check(self._L.ospf_plan_variant(self._h, flags, nh_words, C.byref(v)))
        return v.value

    def plan(self, nh_words: int, flags: int = 0, max_ignored: int = 0,
             n_roots: int = 0xFFFFFFFF, max_root_neighbors: int = 0) -> dict:
        p = N.ospf_plan_info()
        self._check(self._L.ospf_plan_n(self._h, flags, nh_words, max_ignored, n_roots,
                                        max_root_neighbors, C.byref(p)))
        return dict(variant=p.variant, block=p.block, lds_bytes=p.lds_bytes, slices=p.slices)

    @property
    def spf_runs(self) -> int:
        return int(self._L.ospf_spf_runs(self._h))

    def run(self, roots: Sequence[int], nh_words: int, *, hop_count: bool = False,
            want_dist: bool = True, want_nh: bool = True, want_digest: bool = False,
            ignore: Optional[Sequence[Sequence[int]]] = None):
        """Synchronous batch. Returns dict with dist [n,V] u32, nh [n,V,W] u32,
        digest [n,3] u64 (only the requested ones)."""
        roots = np.ascontiguousarray(roots, np.uint32)
        n, V, W = roots.size, self.V, nh_words
        flags = (N.OSPF_HOP_COUNT if hop_count else 0) | \
            (N.OSPF_WANT_DIST if want_dist else 0) | (N.OSPF_WANT_NH if want_nh else 0) | \
            (N.OSPF_WANT_DIGEST if want_digest else 0)
        dist = np.zeros((n, V), np.uint32) if want_dist else None
        nh = np.zeros((n, V, W), np.uint32) if want_nh else None
        dig = np.zeros((n, 3), np.uint64) if want_digest else None
        ig_ref = None
        if ignore is not None:
            off = np.zeros(n + 1, np.uint32)
            off[1:] = np.cumsum([len(x) for x in ignore])
            ids = np.ascontiguousarray(np.concatenate(
                [np.sort(np.asarray(x, np.uint32)) for x in ignore]) if off[-1] else
                np.zeros(1, np.uint32), np.uint32)
            ig = N.ospf_ignore(off.ctypes.data, ids.ctypes.data)
            ig_ref = (C.byref(ig), off, ids)
        self._check(self._L.ospf_sssp_batch(
            self._h, roots.ctypes.data, n, ig_ref[0] if ig_ref else None, flags, W,
            dist.ctypes.data if dist is not None else None,
            nh.ctypes.data if nh is not None else None,
            dig.ctypes.data if dig is not None else None))
        out = {}
        if want_dist:
            out["dist"] = dist
        if want_nh:
            out["nh"] = nh
        if want_digest:
            out["digest"] = dig
        return out

    def run_dev(self, d_roots: int, n_roots: int, nh_words: int, *, flags: int,
                d_dist: int = 0, d_nh: int = 0, d_digest: int = 0, stream: int = 0,
                d_ign_off: int = 0, d_ign_ids: int = 0, max_ignored: int = 0,
                max_root_neighbors: int = 0) -> None:
        """Queue a device-resident batch (raw device pointers) on `stream`.
        max_root_neighbors: optional bound on the roots' distinct neighbour
        counts (sizes the multi-source BFS; 0 = 32 * nh_words)."""
        b = N.ospf_batch(d_roots, n_roots, d_ign_off or None, d_ign_ids or None, max_ignored,
                         flags, nh_words, max_root_neighbors, d_dist or None, d_nh or None,
                         d_digest or None)
        self._check(self._L.ospf_run_batch_dev(self._h, C.byref(b), stream or None))

    @property
    def lev_pitch(self) -> int:
        """Bytes per level row for levels_dev / nh_derive_dev (V rounded up to 16)."""
        return (self.V + 15) // 16 * 16

    def levels_dev(self, d_roots: int, n: int, d_lev: int, *, d_dist: int = 0,
                   d_lev_digest: int = 0, hop_count: bool = False, stream: int = 0,
                   lev_pitch: int = 0) -> None:
        """Derive phase 1 (ospf_levels_dev): dist rows [n][V] (optional), byte
        level rows [n][lev_pitch] and the distance part of each run's digest
        (optional, [n][3] u64) of the n device roots."""
        self._check(self._L.ospf_levels_dev(self._h, d_roots, n,
                                            N.OSPF_HOP_COUNT if hop_count else 0,
                                            d_dist or None, d_lev, lev_pitch or self.lev_pitch,
                                            d_lev_digest or None, stream or None))

    def nh_derive_dev(self, d_roots: int, n: int, nh_words: int, d_lev: int, d_pos: int,
                      d_nh: int, *, d_lev_digest: int = 0, d_digest: int = 0,
                      max_root_neighbors: int = 0, stream: int = 0, lev_pitch: int = 0) -> None:
        """Derive phase 2 (ospf_nh_derive_dev): next-hop rows [n][V][nh_words]
        (+ digests, completing d_lev_digest's parts) from level rows;
        d_pos[v] = level row of node v."""
        self._check(self._L.ospf_nh_derive_dev(self._h, d_roots, n, nh_words, max_root_neighbors,
                                               d_lev, lev_pitch or self.lev_pitch, d_pos,
                                               d_lev_digest or None, d_nh, d_digest or None,
                                               stream or None))

    def wderive_dev(self, d_roots: int, n: int, d_src: int, d_pos: int, d_dist: int, *,
                    src_pitch: int = 0, d_nh: int = 0, d_digest: int = 0,
                    max_root_neighbors: int = 0, hop_count: bool = False,
                    stream: int = 0) -> None:
        """Weighted derive (ospf_wderive_dev): dist rows [n][V], one-word
        next-hop rows [n][V] and digests of n leaf roots (<= 32 distinct
        neighbours) from their neighbours' distance rows
        (d_src + d_pos[v] * src_pitch words)."""
        self._check(self._L.ospf_wderive_dev(self._h, d_roots, n,
                                             N.OSPF_HOP_COUNT if hop_count else 0,
                                             max_root_neighbors, d_src, src_pitch or self.V,
                                             d_pos, d_dist, d_nh or None, d_digest or None,
                                             stream or None))

    def cover_prepare(self, leaf_mask) -> None:
        """ospf_cover_prepare: contracted graph of the cover (nodes outside the
        independent leaf set, leaf_mask[V] bool) for cover_dist_dev."""
        m = np.ascontiguousarray(leaf_mask, np.uint8)
        self._check(self._L.ospf_cover_prepare(self._h, m.ctypes.data))

    def cover_dist_dev(self, d_roots: int, n: int, d_dist: int, stream: int = 0) -> None:
        """ospf_cover_dist_dev: dist rows [n][V] of n cover roots (node ids)."""
        self._check(self._L.ospf_cover_dist_dev(self._h, d_roots, n, d_dist, stream or None))

    def wderive_wide_dev(self, d_roots: int, n: int, nh_words: int, d_src: int, d_pos: int,
                         d_nh: int, *, src_pitch: int = 0, d_digest: int = 0,
                         hop_count: bool = False, stream: int = 0) -> None:
        """ospf_wderive_wide_dev: next-hop rows [n][V][nh_words] (<= 4 words)
        + digests of n roots from their own and their neighbours' dist rows."""
        self._check(self._L.ospf_wderive_wide_dev(self._h, d_roots, n,
                                                  N.OSPF_HOP_COUNT if hop_count else 0, nh_words,
                                                  d_src, src_pitch or self.V, d_pos, d_nh,
                                                  d_digest or None, stream or None))

    def ksp2(self, src: int, dsts: Sequence[int], path_cap: int = 512):
        """getKthPaths(src, d, 1) and (src, d, 2) for every d (ospf_ksp2_run).
        Returns (k1, k2, status): per destination a list of paths (lists of
        link ids, src -> dst) or None where status says the engine's budget
        was exceeded, and the status words."""
        dsts = np.ascontiguousarray(dsts, np.uint32)
        n = dsts.size
        k1 = np.zeros((max(n, 1), path_cap), np.uint32)
        k2 = np.zeros_like(k1)
        st = np.zeros(max(n, 1), np.uint32)
        a = N.ospf_ksp2(src, dsts.ctypes.data, n, path_cap, k1.ctypes.data, k2.ctypes.data,
                        st.ctypes.data)
        self._check(self._L.ospf_ksp2_run(self._h, C.byref(a)))
        return (decode_paths(k1[:n], st[:n], N.OSPF_KSP_OVF1),
                decode_paths(k2[:n], st[:n], N.OSPF_KSP_OVF2 | N.OSPF_KSP_OVF1), st[:n])

    def ksp2_stats(self) -> dict:
        """ospf_ksp2_stats: k = 2 runs by the decremental kernel, runs sent to
        the full masked reruns, affected nodes summed (since open)."""
        out = np.zeros(3, np.uint64)
        self._check(self._L.ospf_ksp2_stats(self._h, out.ctypes.data))
        return {"decremental": int(out[0]), "full_reruns": int(out[1]), "affected": int(out[2])}

    def ksp2_dev(self, src: int, d_dsts: int, n: int, path_cap: int, d_k1: int, d_k2: int,
                 d_status: int, stream: int = 0) -> None:
        a = N.ospf_ksp2(src, d_dsts, n, path_cap, d_k1, d_k2, d_status)
        self._check(self._L.ospf_ksp2_dev(self._h, C.byref(a), stream or None))

    def update_links(self, updates, version: int) -> None:
        """updates: iterable of (link_id, up, metric_lo, metric_hi)."""
        ups = list(updates)
        arr = (N.ospf_link_update * max(len(ups), 1))(*[N.ospf_link_update(*u) for u in ups])
        self._check(self._L.ospf_update_links(self._h, arr, len(ups), version))

    def update_rows(self, csr: Dict[str, np.ndarray], rows, version: int) -> None:
        """ospf_update_rows: links added / removed in place; `csr` is the
        whole CSR after the change, `rows` the nodes whose rows changed."""
        s, keep = csr_struct(csr)
        r = np.ascontiguousarray(rows, np.uint32)
        self._check(self._L.ospf_update_rows(self._h, C.byref(s), r.ctypes.data if r.size else None,
                                             r.size, version))

    def update_nodes(self, nodes, no_transit, version: int) -> None:
        n = np.ascontiguousarray(nodes, np.uint32)
        t = np.ascontiguousarray(no_transit, np.uint8)
        self._check(self._L.ospf_update_nodes(self._h, n.ctypes.data, t.ctypes.data, n.size,
                                              version))

    def affected(self, d_dist: int, n_roots: int, changes, d_out: int, flags: int = 0,
                 stream: int = 0) -> None:
        """changes: iterable of ospf_change field tuples
        (kind, a, b, up0, w_ab0, w_ba0, up1, w_ab1, w_ba1)."""
        ch = list(changes)
        arr = (N.ospf_change * max(len(ch), 1))(*[N.ospf_change(*c) for c in ch])
        self._check(self._L.ospf_affected_roots(self._h, d_dist, n_roots, flags, arr, len(ch),
                                                d_out, stream or None))

    def repair(self, d_roots: int, n: int, nh_words: int, d_dist: int, d_nh: int, changes,
               d_status: int, flags: int = 0, stream: int = 0) -> None:
        """ospf_repair_runs: fix finished rows in place after a patch; d_status
        [n] u32 = 1 where the run must be re-run."""
        ch = list(changes)
        arr = (N.ospf_change * max(len(ch), 1))(*[N.ospf_change(*c) for c in ch])
        self._check(self._L.ospf_repair_runs(self._h, d_roots, n, flags, nh_words, d_dist, d_nh,
                                             arr, len(ch), d_status, stream or None))

    def sync(self, stream: int = 0) -> None:
        self._check(self._L.ospf_sync(self._h, stream or None))

    def links_mask(self, link_ids, version: int) -> None:
        ids = np.ascontiguousarray(link_ids, np.uint32)
        self._check(self._L.ospf_links_mask(self._h, ids.ctypes.data, ids.size, version))

    def links_unmask(self) -> None:
        self._check(self._L.ospf_links_unmask(self._h))

    def sweep(self, **kw) -> "Sweep":
        return Sweep(self, **kw)

    PROBES = {"stream": 0, "rows_chunk": 1, "rows_group": 2, "rows_walk": 3}

    def probe_store(self, pattern: str, V: int, rows: int, group: int = 48, ctiles: int = 6,
                    reps: int = 3) -> np.ndarray:
        """ospf_probe_store: ms per launch writing 2 * rows * V * 4 bytes with
        16-B non-temporal stores (box calibration for the roofline)."""
        out = np.zeros(reps, np.float32)
        self._check(self._L.ospf_probe_store(self._h, self.PROBES[pattern], V, rows, group,
                                             ctiles, reps, out.ctypes.data))
        return out


class Sweep:
    """All-sources sweep (ospf_sweep_*): runSpf for every node of the graph,
    or for part `part` of `n_parts` of the root partition; the library owns
    the path, the width classes, their streams, the row buffers and the HIP
    graph one run replays. ``run(stream)`` queues one sweep."""

    def __init__(self, engine: "Engine", *, hop_count: bool = False, mode: str = "auto",
                 part: int = 0, n_parts: int = 1, hip_graph: bool = True, defer: bool = False,
                 early_start: bool = False, _handle=None):
        self._L = N.engine()
        self.engine = engine
        if _handle is not None:  # a part of an ospf_msweep (owned by it)
            self._h, self._owned = _handle, False
        else:
            # defer: no eager run at create (hip_graph must be off): the
            # first run() is the first run (OSPF_SWEEP_DEFER)
            # early_start (with defer): the first run's serial prefix is
            # queued while the plan is built (OSPF_SWEEP_EARLY_START)
            o = N.ospf_sweep_opts((N.OSPF_HOP_COUNT if hop_count else 0) |
                                  (N.OSPF_SWEEP_DEFER if defer else 0) |
                                  (N.OSPF_SWEEP_EARLY_START if early_start else 0),
                                  N.SWEEP_MODES[mode],
                                  part, n_parts, int(hip_graph and not defer))
            h = C.c_void_p()
            rc = self._L.ospf_sweep_create(engine._h, C.byref(o), C.byref(h))
            if rc != 0:
                raise EngineError(rc, self._L.ospf_last_error(engine._h).decode())
            self._h, self._owned = h, True
        gi = N.ospf_sweep_info()
        self._check(self._L.ospf_sweep_get_info(self._h, C.byref(gi)))
        self.mode = N.SWEEP_MODE_NAMES[gi.mode]
        self.n_roots = int(gi.n_roots)
        self.n_rows = int(gi.n_rows)
        self.n_launches = int(gi.n_launches)
        self.hip_graph = bool(gi.hip_graph)
        self.max_nh_words = int(gi.max_nh_words)
        self.device_bytes = int(gi.device_bytes)
        self.step_compulsory_bytes = int(gi.step_compulsory_bytes)
        self.step_traversed_edges = int(gi.step_traversed_edges)
        r = np.zeros(max(1, self.n_roots), np.uint32)
        self._check(self._L.ospf_sweep_roots(self._h, r.ctypes.data))
        self.roots = r[: self.n_roots]

    def close(self):
        if getattr(self, "_h", None) and self._owned:
            self._L.ospf_sweep_destroy(self._h)
        self._h = None

    __del__ = close

    def _check(self, rc: int):
        if rc != 0:
            raise EngineError(rc, self._L.ospf_sweep_last_error(self._h).decode())

    def run(self, stream: int = 0) -> None:
        self._check(self._L.ospf_sweep_run(self._h, stream or None))

    def digests_dev(self, d_out: int, stream: int = 0) -> None:
        """Digests of the owned roots (roots order) into device memory [n][3] u64."""
        self._check(self._L.ospf_sweep_digests(self._h, d_out, stream or None))

    def poison(self, stream: int = 0) -> None:
        self._check(self._L.ospf_sweep_poison(self._h, stream or None))

    def row(self, root: int):
        """(device dist row pointer, device next-hop row pointer, next-hop words)."""
        d, nh, w = C.c_void_p(), C.c_void_p(), C.c_uint32()
        self._check(self._L.ospf_sweep_row(self._h, int(root), C.byref(d), C.byref(nh),
                                           C.byref(w)))
        return d.value, nh.value, int(w.value)

    def rows(self, roots: Sequence[int], nh_words: int = 0):
        """Host copies of owned roots' rows: dist [n, V] u32, nh [n, V, W] u32
        (W = nh_words or the widest of the roots)."""
        roots = np.ascontiguousarray(roots, np.uint32)
        V = self.engine.V
        W = nh_words or max([self.row(r)[2] for r in roots.tolist()] or [1])
        dist = np.zeros((roots.size, V), np.uint32)
        nh = np.zeros((roots.size, V, W), np.uint32)
        self._check(self._L.ospf_sweep_copy_rows(self._h, roots.ctypes.data, roots.size, W,
                                                 dist.ctypes.data, nh.ctypes.data))
        return dist, nh

    def profile(self, reps: int = 3):
        """Every launch unit timed alone on its stream -> list of dicts."""
        cap = max(1, self.n_launches)
        arr = (N.ospf_sweep_launch * cap)()
        self._check(self._L.ospf_sweep_profile(self._h, reps, arr, cap))
        return [dict(name=a.name.decode(), kernel=a.kernel.decode(), n_roots=int(a.n_roots),
                     nh_words=int(a.nh_words), compulsory_bytes=int(a.compulsory_bytes),
                     ms_median=float(a.ms_median), ms_min=float(a.ms_min))
                for a in arr[: self.n_launches]]

    def graph_memsets(self):
        """Diagnostic: the captured graph's memset nodes -> (count, with a
        destination outside every live allocation, inside the sweep's own
        blocks); see ospf_sweep_graph_memsets."""
        a, b, c = C.c_uint32(), C.c_uint32(), C.c_uint32()
        self._check(self._L.ospf_sweep_graph_memsets(self._h, C.byref(a), C.byref(b), C.byref(c)))
        return int(a.value), int(b.value), int(c.value)


class Multi:
    """Several devices behind one handle (ospf_multi_*): the graph replicated,
    sweeps partitioned by device slot, digests gathered by peer copies."""

    def __init__(self, devices: Sequence[int]):
        self._L = N.engine()
        devs = np.ascontiguousarray(devices, np.int32)
        h = C.c_void_p()
        rc = self._L.ospf_multi_open(devs.ctypes.data, devs.size, C.byref(h))
        if rc != 0:
            raise EngineError(rc, f"ospf_multi_open({list(devices)}) failed")
        self._h = h
        self.n = int(self._L.ospf_multi_size(h))
        self.V = 0

    def close(self):
        if getattr(self, "_h", None):
            self._L.ospf_multi_close(self._h)
            self._h = None

    __del__ = close

    def _check(self, rc: int):
        if rc != 0:
            raise EngineError(rc, self._L.ospf_multi_last_error(self._h).decode())

    def load(self, csr: Dict[str, np.ndarray], version: int = 1) -> None:
        s, keep = csr_struct(csr)
        self._check(self._L.ospf_multi_load_graph(self._h, C.byref(s), version))
        self.V = int(s.n_nodes)


class MultiSweep:
    """ospf_msweep_*: one sweep part per device slot of a Multi."""

    def __init__(self, multi: Multi, *, hop_count: bool = False, mode: str = "auto",
                 hip_graph: bool = True):
        self._L = N.engine()
        self.multi = multi
        o = N.ospf_sweep_opts(N.OSPF_HOP_COUNT if hop_count else 0, N.SWEEP_MODES[mode], 0, 0,
                              int(hip_graph))
        h = C.c_void_p()
        rc = self._L.ospf_msweep_create(multi._h, C.byref(o), C.byref(h))
        if rc != 0:
            raise EngineError(rc, self._L.ospf_multi_last_error(multi._h).decode())
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            self._L.ospf_msweep_destroy(self._h)
            self._h = None

    __del__ = close

    def run(self) -> None:
        self.multi._check(self._L.ospf_msweep_run(self._h))

    def digests(self) -> np.ndarray:
        out = np.zeros((self.multi.V, 3), np.uint64)
        self.multi._check(self._L.ospf_msweep_digests(self._h, out.ctypes.data))
        return out

    @property
    def gather_backend(self) -> str:
        """'rccl' (one ncclAllGather of the parts' digests) or 'peer'."""
        return "rccl" if self._L.ospf_msweep_gather_backend(self._h) else "peer"

    def owner(self, root: int) -> int:
        s = C.c_uint32()
        self.multi._check(self._L.ospf_msweep_owner(self._h, int(root), C.byref(s)))
        return int(s.value)

    def part_roots(self, slot: int) -> np.ndarray:
        h = self._L.ospf_msweep_part(self._h, slot)
        gi = N.ospf_sweep_info()
        self._L.ospf_sweep_get_info(h, C.byref(gi))
        r = np.zeros(max(1, gi.n_roots), np.uint32)
        self._L.ospf_sweep_roots(h, r.ctypes.data)
        return r[: gi.n_roots]
