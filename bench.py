#!/usr/bin/env python3
"""Benchmark: all-sources SPF + ECMP next-hops on the 100k-node fabric.

BASELINE.json metric: "all-sources SPF/sec + GTEPS on 100k-node fabric
topology at 1/2/4/8 GPUs". A *step* = one batch of roots per GPU run through
the engine's device API (ospf_sssp_batch_dev): per-root distance rows,
next-hop bitset rows and digests written to HBM, then (N > 1) the 24-B
per-root digest records all-gathered over RCCL. Roots sweep a fixed
permutation of every node (all sources); each step launches one kernel per
next-hop width class (rack / fabric / spine switches), each on its own HIP
stream. Ranks shard the roots with no data-path collective: scaling "weak".

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
       torchrun --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
                --master-port P bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

import torch  # first: the engine shares torch's HIP runtime (device buffers, events)

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from openr_amd import _native as N  # noqa: E402
from openr_amd import shard  # noqa: E402
from openr_amd import topology as T  # noqa: E402
from openr_amd.engine import Engine  # noqa: E402
from openr_amd.linkstate import LinkState  # noqa: E402

METRIC = "all-sources SPF/sec + GTEPS on 100k-node fabric topology at 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def build_topology(name: str):
    if name == "fabric100k":
        return T.fabric(pods=1781, planes=8), "F100k fabric pods=1781 planes=8 (unit metric)"
    if name == "fabric10k":
        return T.fabric(pods=173, planes=8), "F10k fabric pods=173 planes=8 (unit metric)"
    if name == "fabric100k-w":
        return (T.fabric(pods=1781, planes=8, weighted_seed=7),
                "F100k fabric pods=1781 planes=8 (metric 1..64, seed 7)")
    if name == "grid31":
        return T.grid(31), "G31 grid 31x31 (unit metric)"
    if name == "mesh1m":
        return T.mesh(1_000_000, seed=42), "M1M random-geometric mesh (metric 1..16)"
    raise SystemExit(f"unknown topology {name}")


def bytes_per_root(V: int, E: int, W: int) -> int:
    """SURVEY.md §8(d) algorithmic bytes of one SPF run: CSR neighbour + weight
    reads, row offsets, dist write, next-hop bitset write."""
    return 8 * E + 4 * (V + 1) + 4 * V + 4 * V * W


def pmc_traffic(profile_dir: str, key: str, roots: int):
    """Measured HBM bytes per launch of the class `key` with `roots` roots from
    the committed per-class rocprofv3 --pmc summary (profiles/<round>/
    pmc_traffic.json, written by scripts/pmc_class_traffic.py: FETCH_SIZE x 2
    (gfx950 correction) + WRITE_SIZE, summed over the class's kernels); None
    when absent or measured at another batch size."""
    path = os.path.join(profile_dir, "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            e = json.load(f).get(key, {})
    except (OSError, ValueError):
        return None
    return e.get("hbm_bytes_per_launch") if e.get("roots_per_launch") == roots else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=16384,
                    help="roots per GPU per step (6 steps sweep all 100k sources of F100k)")
    ap.add_argument("--topology", default="fabric100k")
    ap.add_argument("--cpu-sample", type=int, default=32)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-nh", action="store_true", help="skip next-hop output (diagnostic)")
    ap.add_argument("--serial-streams", action="store_true", help="one stream for all classes")
    ap.add_argument("--root-order", choices=["auto", "locality", "random"], default="auto",
                    help="sweep order within a width class: grouped by smallest neighbour "
                         "(multi-source batches share frontiers), the random permutation, or "
                         "auto = grouped for single-word classes only (measured: grouping "
                         "wide roots makes their per-pass next-hop planes denser and slower)")
    ap.add_argument("--profile-dir", default=os.path.join(ROOT, "profiles", "r01"))
    ap.add_argument("--iso-reps", type=int, default=3,
                    help="isolated launches per class for the roofline (after the timed steps)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist_on = world > 1
    if dist_on:
        torch.distributed.init_process_group("nccl", device_id=dev)

    t0 = time.time()
    stream, desc = build_topology(args.topology)
    ls = LinkState(device=local, stream=stream)
    csr = ls.csr()
    names = ls.node_names()
    eng = Engine(local)
    eng.load(csr)
    V, E = eng.V, int(csr["col"].size)
    props = torch.cuda.get_device_properties(local)
    log(f"[rank {rank}] {props.name} CUs={props.multi_processor_count} "
        f"{desc}: V={V} E_dir={E} setup {time.time() - t0:.1f}s")

    flags = N.OSPF_WANT_DIST | N.OSPF_WANT_DIGEST | (0 if args.no_nh else N.OSPF_WANT_NH)
    perm = np.random.default_rng(0x5EED).permutation(V).astype(np.uint32)
    nbrs = shard.distinct_neighbors(csr["row_ptr"], csr["col"])
    words = np.maximum(1, (nbrs + 31) // 32)
    key = shard.first_neighbor(csr["row_ptr"], csr["col"]) if args.root_order != "random" \
        else None
    classes = shard.make_classes(perm, words, args.batch, key,
                                 max_grouped_words=1 if args.root_order == "auto" else None)
    B = sum(c.per_step for c in classes)
    for c in classes:
        n = c.per_step
        x = c.extra
        x["max_nbrs"] = int(max(1, nbrs[c.roots].max()))  # engine hint: sizes bit-planes
        x["plan"] = eng.plan(c.nh_words, flags, n_roots=n, max_root_neighbors=x["max_nbrs"])
        x["d_all"] = torch.from_numpy(c.roots.astype(np.int32)).to(dev)
        x["roots"] = torch.empty(n, dtype=torch.int32, device=dev)
        x["dist"] = torch.empty((n, V), dtype=torch.int32, device=dev)
        x["nh"] = None if args.no_nh else torch.empty((n, V, c.nh_words), dtype=torch.int32,
                                                      device=dev)
        x["dig"] = torch.empty((n, 3), dtype=torch.int64, device=dev)
        x["stream"] = torch.cuda.current_stream() if args.serial_streams else \
            torch.cuda.Stream(device=dev)
        x["ev"] = []
    dig_all = torch.empty((B, 3), dtype=torch.int64, device=dev)
    main_s = torch.cuda.current_stream()
    order = sorted(classes, key=lambda c: -c.nh_words)  # longest runs first

    def step(i: int, timed: bool):
        ready = torch.cuda.Event()
        ready.record(main_s)  # the previous step's digest copies are queued on main_s
        done = []
        for c in order:
            x, n, m = c.extra, c.per_step, c.roots.size
            cs = x["stream"]
            with torch.cuda.stream(cs):
                cs.wait_event(ready)
                start = ((i * world + rank) * n) % m  # == shard.step_roots on the device
                idx = (torch.arange(n, device=dev) + start) % m
                torch.index_select(x["d_all"], 0, idx, out=x["roots"])
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record(cs)
                eng.run_dev(x["roots"].data_ptr(), n, c.nh_words, flags=flags,
                            d_dist=x["dist"].data_ptr(),
                            d_nh=x["nh"].data_ptr() if x["nh"] is not None else 0,
                            d_digest=x["dig"].data_ptr(), stream=cs.cuda_stream,
                            max_root_neighbors=x["max_nbrs"])
                ev[1].record(cs)
            done.append(ev[1])
            if timed:
                x["ev"].append(ev)
        for e in done:
            main_s.wait_event(e)
        off = 0
        for c in classes:
            dig_all[off:off + c.per_step].copy_(c.extra["dig"])
            off += c.per_step
        if dist_on:
            shard.gather_digests(dig_all)

    for i in range(args.warmup):
        step(i, False)
    torch.cuda.synchronize()
    eng.sync(main_s.cuda_stream)
    if dist_on:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i, True)
    torch.cuda.synchronize()
    if dist_on:
        torch.distributed.barrier()
    dt = time.perf_counter() - t_start
    eng.sync(main_s.cuda_stream)  # raises if the device error word was set
    if dist_on:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t.item())

    roots_total = world * B * args.steps
    spf_s = roots_total / dt
    gteps = roots_total * E / dt / 1e9

    # roofline. The classes overlap on their streams inside the timed steps,
    # so each class is then timed ALONE (not part of `value`): R launches on
    # one stream bracketed by HIP events on that stream. The dominant class is
    # the one with the largest share of a step's device time. A multi-source
    # class launch is a sequence of kernels (init, level/settle pairs, rows);
    # its events bracket the whole sequence, and profiles/<round>/ holds the
    # rocprofv3 per-kernel summary whose per-class sums it matches.
    iso_s = torch.cuda.Stream(device=dev)
    for c in classes:
        x = c.extra
        ms = []
        with torch.cuda.stream(iso_s):
            for _ in range(args.iso_reps + 1):
                a_, b_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a_.record(iso_s)
                eng.run_dev(x["roots"].data_ptr(), c.per_step, c.nh_words, flags=flags,
                            d_dist=x["dist"].data_ptr(),
                            d_nh=x["nh"].data_ptr() if x["nh"] is not None else 0,
                            d_digest=x["dig"].data_ptr(), stream=iso_s.cuda_stream,
                            max_root_neighbors=x["max_nbrs"])
                b_.record(iso_s)
                b_.synchronize()
                ms.append(a_.elapsed_time(b_))
        x["iso_ms"] = float(np.median(ms[1:]))
        x["ms"] = [a_.elapsed_time(b_) for a_, b_ in x["ev"]]
    eng.sync(iso_s.cuda_stream)

    def class_roofline(c):
        x, p = c.extra, c.extra["plan"]
        alg = c.per_step * bytes_per_root(V, E, c.nh_words)
        ach = alg / (x["iso_ms"] / 1e3) / 1e9
        tr = pmc_traffic(args.profile_dir, f"variant{p['variant']}_W{c.nh_words}", c.per_step)
        return {"nh_words": c.nh_words, "roots_per_launch": c.per_step,
                "isolated_launch_ms": round(x["iso_ms"], 3),
                "achieved": round(ach, 1), "frac": round(ach / HBM_PEAK_GBS, 4),
                "traffic": tr,
                "traffic_GBs": round(tr / (x["iso_ms"] / 1e3) / 1e9, 1) if tr else None}

    dom = max(classes, key=lambda c: c.extra["iso_ms"])
    dr = class_roofline(dom)
    p = dom.extra["plan"]
    roofline = {
        "bound": "hbm", "achieved": dr["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": dr["frac"], "traffic": dr["traffic"],
        "kernel": (f"multi-source BFS class launch (variant 5, nh_words {dom.nh_words}: "
                   f"msbfs init + level/settle pairs + rows kernels)")
        if p["variant"] == 5 else
        f"spf_bfs_kernel (variant {p['variant']}, nh_words {dom.nh_words})"
        if p["variant"] >= 3 else f"spf_run_kernel (variant {p['variant']})",
        "block": p["block"], "roots_per_launch": dom.per_step,
        "bytes_per_root": bytes_per_root(V, E, dom.nh_words),
        "avg_launch_ms": dr["isolated_launch_ms"],
        "traffic_GBs": dr["traffic_GBs"],
        "edges_per_s_per_launch": round(dom.per_step * E / (dom.extra["iso_ms"] / 1e3), 1),
        "classes": [class_roofline(c) for c in classes],
        "note": "achieved = roots x SURVEY 8(d) bytes_root (8E + 8V + 4VW: every root scanning "
                "the CSR) / isolated launch time; 64 roots share each CSR scan, so achieved "
                "can exceed the HBM peak; traffic = measured HBM bytes per launch (rocprofv3 "
                "FETCH_SIZE x2 + WRITE_SIZE, profiles/<round>/pmc_traffic.json)",
    }

    cpu = parity = None
    if rank == 0 and world == 1 and not args.no_cpu:
        from oracle import Oracle  # CPU baseline leg only (reference-shaped restatement)
        sample_ids = perm[: args.cpu_sample]
        sample = [names[i] for i in sample_ids]
        o = Oracle(stream)
        t1 = time.perf_counter()
        cd = o.digests(sample, threads=args.cpu_threads)
        ct = time.perf_counter() - t1
        cpu = {"value": round(len(sample) / ct, 4), "unit": "SPF/s", "cores": args.cpu_threads,
               "kind": "port",
               "sample": f"{len(sample)} roots (permutation seed 0x5eed) of the same topology, "
                         f"reference-shaped runSpf restatement (oracle/), {args.cpu_threads} "
                         f"threads, {ct:.2f}s"}
        gd = eng.run(sample_ids, int(words[sample_ids].max()), want_dist=False, want_nh=False,
                     want_digest=True)["digest"]
        parity = bool(np.array_equal(gd, cd))

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(spf_s, 2), "unit": "SPF/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u32", "data": "synthetic",
            "gteps": round(gteps, 3),
            "config": {
                "workload": desc + " all-sources SPF + ECMP next-hop bitsets (dist + next-hop "
                                   "rows written to HBM, per-root digests)",
                "n_nodes": V, "n_directed_edges": E, "roots_per_step_per_gpu": B,
                "root_classes": [{"nh_words": c.nh_words, "roots_per_step": c.per_step,
                                  **{k: c.extra["plan"][k] for k in ("variant", "slices",
                                                                     "block")},
                                  "avg_launch_ms": round(float(np.mean(c.extra["ms"])), 3),
                                  "isolated_launch_ms": round(c.extra["iso_ms"], 3)}
                                 for c in classes],
                "parallelism": f"root-sharded x{world}" +
                               (", RCCL all_gather of 24-B digests" if dist_on else "")},
            "roofline": roofline, "cpu_baseline": cpu, "parity_vs_cpu_sample": parity,
        }
        print(json.dumps(line), flush=True)
    if dist_on:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
