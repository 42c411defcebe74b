#!/usr/bin/env python3
"""Production call stack A at F100k:
what Decision runs per route rebuild on one node --

    getSpfResult(myNodeName)      (LinkState.cpp:821-831; engine SPF + host
                                   SpfResult rebuild, link_state.cpp buildResult)
    -> route build                (SpfSolver::buildRouteDb, SpfSolver.cpp:460-646:
                                   every node's loopback prefix + MPLS node /
                                   adjacency labels, odl::SpfSolver)

timed through odl::LinkState on the MI355X, phase by phase (ODL_SPF_TIMING
lines from libopenr_decision), cold (snapshot + device load) and warm, and
after a link-metric event and a [LINK DOWN] / [LINK UP] pair (adjacency
withdrawn and restored, patched in place: apply, getSpfResult(me), an
all-sources re-sweep) with incremental patching off / on; next to the CPU
restatement of runSpf on the same root (oracle/, reference-shaped).

Usage: python scripts/prod_callstack.py [--pods 1781] > out.json
"""
from __future__ import annotations

import argparse
import json
import os
import re
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["ODL_SPF_TIMING"] = "1"
os.environ.setdefault("OSPF_SWEEP_TIMING", "1")  # sweep + graph-load phases
os.environ.setdefault("ODL_SNAP_TIMING", "1")    # CSR snapshot phases

import torch  # noqa: E402,F401  (one HIP runtime for torch and the engine)

from openr_amd import topology as T  # noqa: E402
from openr_amd.adjdb import AdjDbStream  # noqa: E402
from openr_amd.linkstate import LinkState  # noqa: E402


class Stderr:
    """Capture the C++ timing lines written to fd 2."""

    def __enter__(self):
        self.f = tempfile.TemporaryFile("w+")
        sys.stderr.flush()
        self.saved = os.dup(2)
        os.dup2(self.f.fileno(), 2)
        return self

    def __exit__(self, *a):
        sys.stderr.flush()
        os.dup2(self.saved, 2)
        os.close(self.saved)
        self.f.seek(0)
        self.text = self.f.read()
        self.f.close()

    def laps(self):
        """OSPF_SWEEP_TIMING's ospf_sweep_create phases -> {phase: ms}"""
        return {k: float(v) for k, v in re.findall(r"sweep_create (.+?) ([0-9.]+) ms", self.text)}

    def snap_laps(self):
        """ODL_SNAP_TIMING's CSR snapshot phases -> {phase: ms}"""
        return {k: float(v) for k, v in re.findall(r"snapshot (.+?) ([0-9.]+) ms", self.text)}

    def values(self, key):
        return [float(x) for x in re.findall(key + r"=([0-9.]+)", self.text)]


def timed(fn):
    with Stderr() as cap:
        t = time.perf_counter()
        out = fn()
        wall = (time.perf_counter() - t) * 1e3
    return out, wall, cap


def progress(msg):
    """a line on the real stderr (fd 2 may be captured by Stderr)"""
    with open("/proc/self/fd/%d" % PROGRESS_FD, "a") as f:
        f.write(f"[{time.strftime('%H:%M:%S')}] {msg}\n")


PROGRESS_FD = os.dup(2)


def main():
    import faulthandler
    trace = os.environ.get("PROD_TRACE_FILE")
    if trace:  # where a stalled step is, every 60 s
        faulthandler.dump_traceback_later(60, repeat=True, file=open(trace, "w"))
    ap = argparse.ArgumentParser()
    ap.add_argument("--pods", type=int, default=1781)
    ap.add_argument("--me", default="3-0-0")
    ap.add_argument("--other", default="3-17-5")
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()
    st = T.fabric(pods=args.pods, planes=8)
    out = {"topology": f"fabric pods={args.pods} planes=8 (unit metric)", "me": args.me}

    def stack(p, me, label):
        progress(f"{label}: getSpfResult")
        _, wall, cap = timed(lambda: p.prefetch([me]))
        rec = {"getSpfResult_wall_ms": round(wall, 3),
               "engine_ms": sum(cap.values("engine_ms")),
               "build_result_ms": sum(cap.values("build_result_ms"))}
        if cap.laps():  # ospf_load_graph phases (a cold call loads the graph)
            rec["engine_laps"] = cap.laps()
        if cap.snap_laps():
            rec["snapshot_laps"] = cap.snap_laps()
        for k in ("open_ms", "load_ms"):  # ensureEngine (ODL_SPF_TIMING)
            if cap.values(k):
                rec["ensure_engine_" + k] = sum(cap.values(k))
        names = p.node_names()
        prefixes = {f"lo-{n}": [[n, "ip", "ecmp", 0, None]] for n in names}
        lines = [f"{pfx}\t{ents[0][0]}:0:0:0:" for pfx, ents in prefixes.items()]
        raw, wall_r, cap_r = timed(lambda: p.route_db_bin_raw([me], lines, 3))
        rec["route_build_ms"] = sum(cap_r.values("build_route_db_ms"))
        rec["route_build_wall_ms_incl_binary_abi"] = round(wall_r, 3)
        rec["route_db_binary_bytes"] = len(raw)
        t = time.perf_counter()
        from openr_amd.linkstate import decode_route_db_bin
        decode_route_db_bin(raw)
        rec["python_decode_of_binary_ms"] = round((time.perf_counter() - t) * 1e3, 1)
        _, wall_t, _ = timed(lambda: p.route_dbs([me], prefixes, binary=False))
        rec["route_build_wall_ms_incl_text_abi_and_python_parse"] = round(wall_t, 3)
        rec["total_ms"] = round(rec["getSpfResult_wall_ms"] + rec["route_build_ms"], 3)
        out[label] = rec
        print(f"{label}: {rec}", file=sys.stderr, flush=True)

    for incremental in (False, True):
        progress(f"ingest incremental={incremental}")
        p = LinkState()
        p.set_incremental(incremental)
        t = time.perf_counter()
        p.apply(st)
        ingest = (time.perf_counter() - t) * 1e3
        tag = "incremental" if incremental else "default"
        out[f"{tag}_ingest_ms"] = round(ingest, 1)
        stack(p, args.me, f"{tag}_cold")      # snapshot + engine open/load + run
        stack(p, args.other, f"{tag}_warm")   # graph resident: run + rebuild
        # a link-metric event on a far link, then the same node's rebuild
        db = [d for d in st.to_dbs() if d.name == "3-900-0"][0]
        db.adjs[0].metric = 3
        ev = AdjDbStream.from_dbs([db])
        _, wall, _ = timed(lambda: p.apply(ev))
        out[f"{tag}_event_apply_ms"] = round(wall, 3)
        stack(p, args.me, f"{tag}_after_event")
        # the metric back to 1: the graph is unit-metric again (one metric-3
        # link makes the whole graph weighted -- the weighted sweep path --
        # which r04's link events measured by accident)
        db.adjs[0].metric = 1
        _, wall, _ = timed(lambda: p.apply(AdjDbStream.from_dbs([db])))
        out[f"{tag}_metric_revert_apply_ms"] = round(wall, 3)
        # [LINK DOWN] / [LINK UP] (LinkState.cpp:632-657): a rack withdraws
        # its adjacency to its pod's first fabric switch, then restores it;
        # each: apply, getSpfResult(me), and a whole all-sources re-sweep
        db = [d for d in st.to_dbs() if d.name == "3-901-0"][0]
        _, wall, cap = timed(lambda: p.prefetch_all())
        out[f"{tag}_all_sources_sweep_before_link_events_ms"] = round(wall, 3)
        out[f"{tag}_all_sources_sweep_before_link_events_create"] = cap.laps()
        t0 = p.topology_stats()
        adj = db.adjs.pop(0)
        for kind in ("link_down", "link_up"):
            if kind == "link_up":
                db.adjs.insert(0, adj)
            ev = AdjDbStream.from_dbs([db])
            _, wall, _ = timed(lambda: p.apply(ev))
            out[f"{tag}_{kind}_apply_ms"] = round(wall, 3)
            _, wall, cap = timed(lambda: p.prefetch([args.me]))
            out[f"{tag}_{kind}_getSpfResult_ms"] = round(wall, 3)
            out[f"{tag}_{kind}_engine_ms"] = sum(cap.values("engine_ms"))
            _, wall, cap = timed(lambda: p.prefetch_all())
            out[f"{tag}_{kind}_all_sources_sweep_ms"] = round(wall, 3)
            out[f"{tag}_{kind}_all_sources_sweep_create"] = cap.laps()
            print(f"{tag} {kind}: apply {out[f'{tag}_{kind}_apply_ms']} ms, getSpfResult "
                  f"{out[f'{tag}_{kind}_getSpfResult_ms']} ms, sweep "
                  f"{out[f'{tag}_{kind}_all_sources_sweep_ms']} ms", file=sys.stderr, flush=True)
        t1 = p.topology_stats()
        out[f"{tag}_link_events_topology_stats"] = {k: t1[k] - t0[k] for k in t1}
        # a steady re-sweep of the same graph version (the sweep is resident)
        # and [NODE DOWN] / [NODE UP]: a rack's database deleted and restored
        # (in place on the host snapshot; the device graph reloads)
        from openr_amd.adjdb import AdjDb
        rack = [d for d in st.to_dbs() if d.name == "3-902-7"][0]
        for kind, ev in (("node_down", AdjDbStream.from_dbs([AdjDb(rack.name, delete=True)])),
                         ("node_up", AdjDbStream.from_dbs([rack]))):
            progress(f"{tag} {kind}")
            _, wall, _ = timed(lambda: p.apply(ev))
            out[f"{tag}_{kind}_apply_ms"] = round(wall, 3)
            _, wall, cap = timed(lambda: p.prefetch([args.me]))
            out[f"{tag}_{kind}_getSpfResult_ms"] = round(wall, 3)
            _, wall, cap = timed(lambda: p.prefetch_all())
            out[f"{tag}_{kind}_all_sources_sweep_ms"] = round(wall, 3)
            out[f"{tag}_{kind}_all_sources_sweep_create"] = cap.laps()
            print(f"{tag} {kind}: apply {out[f'{tag}_{kind}_apply_ms']} ms, getSpfResult "
                  f"{out[f'{tag}_{kind}_getSpfResult_ms']} ms, sweep "
                  f"{out[f'{tag}_{kind}_all_sources_sweep_ms']} ms", file=sys.stderr, flush=True)
        out[f"{tag}_node_patches"] = p.node_patches
        del p
    if not args.no_cpu:
        from oracle import Oracle  # CPU restatement, same root
        o = Oracle(st)
        t = time.perf_counter()
        txt = o.spf_text(args.me, True)
        out["cpu_runSpf_ms"] = round((time.perf_counter() - t) * 1e3, 3)
        out["cpu_runSpf_note"] = ("reference-shaped runSpf restatement (oracle/), one thread, "
                                  f"result text {len(txt)} bytes")
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
