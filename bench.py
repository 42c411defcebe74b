#!/usr/bin/env python3
"""Benchmark: all-sources SPF + ECMP next hops on the 100k-node fabric.

BASELINE.json metric: "all-sources SPF/sec + GTEPS on 100k-node fabric
topology at 1/2/4/8 GPUs". A *step* = one all-sources sweep: every node of
the topology is the root of one SPF run (LinkState::runSpf,
openr/decision/LinkState.cpp:836-911) whose distance row and next-hop bitset
row are written to HBM, plus a 24-B digest per run. The roots are split
over the ranks (one process per GPU, contiguous slices of each next-hop width
class), so the total work per step is fixed: scaling "strong". Each rank
launches one engine call per width class (rack / fabric / spine switches),
each on its own HIP stream; for N > 1 the digest records are all-gathered
over RCCL. The timed steps' own digests of the CPU-sample roots are checked
against the CPU restatement (`parity_vs_cpu_sample`).

Other topologies (parity / side benches, not the headline): fabric10k,
fabric100k-w and fabric10k-w (metrics 1..64, seed 7: weighted derive mode,
wderive_main), grid31, mesh1m (8,192 sampled roots).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--topology T]
       torchrun --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \\
                --master-port P bench.py --gpus N ...
Profiling mode (one class alone, R launches on one stream, no JSON line):
       python bench.py --class-only W --reps R
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
SEED = 0x5EED


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def build_topology(name: str):
    """-> (stream, description, weighted, default root count (0 = all))"""
    if name == "fabric100k":
        return T.fabric(pods=1781, planes=8), "F100k fabric pods=1781 planes=8 (unit metric)", \
            False, 0
    if name == "fabric10k":
        return T.fabric(pods=173, planes=8), "F10k fabric pods=173 planes=8 (unit metric)", False, 0
    if name == "fabric100k-w":
        return (T.fabric(pods=1781, planes=8, weighted_seed=7),
                "F100k fabric pods=1781 planes=8 (metric 1..64, seed 7)", True, 0)
    if name == "fabric10k-w":
        return (T.fabric(pods=173, planes=8, weighted_seed=7),
                "F10k fabric pods=173 planes=8 (metric 1..64, seed 7)", True, 0)
    if name == "grid31":
        return T.grid(31), "G31 grid 31x31 (unit metric)", False, 0
    if name == "mesh1m":
        return T.mesh(1_000_000, seed=42), "M1M random-geometric mesh (metric 1..16)", True, 8192
    raise SystemExit(f"unknown topology {name}")


def bytes_per_root(V: int, E: int, W: int) -> int:
    """SURVEY.md §8(d) model of one SPF run: CSR neighbour + weight reads,
    row offsets, dist write, next-hop bitset write. Every root is charged a
    full CSR scan, which batched traversals do not make (alg_equiv only)."""
    return 8 * E + 4 * (V + 1) + 4 * V + 4 * V * W


def compulsory_bytes(V: int, E: int, W: int, n: int, variant: int, npass: int,
                     weighted: bool) -> int:
    """Bytes a launch of n runs cannot avoid: the dist + next-hop rows it
    writes (4V(1 + W) per run) plus the CSR reads its traversals need at
    least once: the multi-source BFS (variant 5) scans neighbour ids + row
    offsets once per 64-root pass (ceil(n / 64) * npass passes); a per-root
    kernel scans them once per run, with both metric arrays when weighted."""
    rows = n * 4 * V * (1 + W)
    if variant == 5:
        scans = -(-n // 64) * npass
        per_scan = 4 * E + 4 * (V + 1)
    else:
        scans = n
        per_scan = (12 if weighted else 4) * E + 4 * (V + 1)
    return rows + scans * per_scan


def pmc_traffic(profile_dir: str, key: str, roots: int):
    """Measured HBM bytes per launch of class `key` with `roots` roots from
    the committed per-class rocprofv3 --pmc summary (profiles/<round>/
    pmc_traffic.json, scripts/pmc_class_traffic.py: FETCH_SIZE x 2 (gfx950
    correction) + WRITE_SIZE, summed over the class's kernels); None when
    absent or measured at another batch size."""
    path = os.path.join(profile_dir, "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            e = json.load(f).get(key, {})
    except (OSError, ValueError):
        return None
    return e.get("hbm_bytes_per_launch") if e.get("roots_per_launch") == roots else None


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_threads() -> int:
    """Host cores this process may use: the affinity mask, capped by
    OMP_NUM_THREADS (the GPU box grants 16 and says so there)."""
    n = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(omp))) if omp and omp.isdigit() else n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=60,
                    help="timed steps (default: a few seconds of timed work at F100k)")
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--topology", default="fabric100k")
    ap.add_argument("--roots", type=int, default=-1,
                    help="roots per step over all GPUs: 0 = every node (all-sources), k = a "
                         "fixed sample of k nodes (seed 0x5eed); default per topology")
    ap.add_argument("--roots-per-gpu", type=int, default=0,
                    help="weak-scaling mode: each rank sweeps this many roots per step")
    ap.add_argument("--cpu-sample", type=int, default=-1,
                    help="roots of the reference-shaped CPU baseline (default 256; 16 on M1M)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = the host cores granted")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-nh", action="store_true", help="skip next-hop output (diagnostic)")
    ap.add_argument("--serial-streams", action="store_true", help="one stream for all classes")
    ap.add_argument("--root-order", choices=["auto", "locality", "random"], default="auto",
                    help="sweep order within a width class: grouped by smallest neighbour "
                         "(multi-source batches share frontiers), the random permutation, or "
                         "auto = grouped for single-word classes only")
    ap.add_argument("--profile-dir", default=os.path.join(ROOT, "profiles", "r02"))
    ap.add_argument("--iso-reps", type=int, default=3,
                    help="isolated launches per class for the roofline (after the timed steps)")
    ap.add_argument("--class-only", type=int, default=0,
                    help="profiling mode: launch only the class with this neighbour capacity "
                         "(8, 16, or 32 x next-hop words)")
    ap.add_argument("--reps", type=int, default=3, help="launches in --class-only mode")
    ap.add_argument("--mode", choices=["auto", "derive", "batch"], default="auto",
                    help="derive: all-sources next hops from neighbour level rows (unit "
                         "metric, every root's neighbours in the sweep); batch: per-class "
                         "engine batches (bit-plane next hops); auto = derive when it applies")
    ap.add_argument("--wide", choices=["derive", "batch"], default="derive",
                    help="derive mode: rows of > 4 next-hop words (spines) from level rows "
                         "(nh_derive_wide_kernel) or on the bit-plane batch path")
    ap.add_argument("--graph", choices=["auto", "on", "off"], default="auto",
                    help="derive mode: capture one step's launches in a HIP graph and replay "
                         "it (auto: on; falls back to eager launches if capture fails)")
    ap.add_argument("--wcover", choices=["spf", "batch"], default="spf",
                    help="weighted all-sources: cover roots by the contracted-graph SPF "
                         "(ospf_cover_dist_dev + ospf_wderive_wide_dev) or per-root batches")
    ap.add_argument("--dist-parity", type=int, default=0,
                    help="N>1: rank 0 checks the gathered digests of the last timed step "
                         "for this many roots against the CPU restatement")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # Multi-rank rehearsal on one GPU (tests/test_gpu_multirank.py): every rank
    # on device 0, gloo for the collectives (RCCL refuses two ranks per GPU).
    if os.environ.get("OPENR_BENCH_SHARE_DEVICE") == "1":
        local = 0
    backend = os.environ.get("OPENR_BENCH_BACKEND", "nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist_on = world > 1
    if dist_on:
        if backend == "nccl":
            torch.distributed.init_process_group("nccl", device_id=dev)
        else:
            torch.distributed.init_process_group(backend)
    coll_dev = dev if backend == "nccl" else torch.device("cpu")

    t0 = time.time()
    stream, desc, weighted, default_roots = build_topology(args.topology)
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
    perm = np.random.default_rng(SEED).permutation(V).astype(np.uint32)
    n_roots = default_roots if args.roots < 0 else args.roots
    derive_ok = (n_roots <= 0 and not weighted and args.roots_per_gpu == 0 and not args.no_nh
                 and not args.class_only and eng.info().unit_metric
                 and int(shard.distinct_neighbors(csr["row_ptr"], csr["col"]).max()) <= 2048)
    if args.mode != "batch" and derive_ok:
        return derive_main(args, eng, csr, names, stream, desc, V, E, world, rank, dist_on, dev,
                           backend, coll_dev)
    wderive_ok = (n_roots <= 0 and not derive_ok and args.roots_per_gpu == 0 and not args.no_nh
                  and not args.class_only)
    if args.mode == "derive" and not (derive_ok or wderive_ok):
        raise SystemExit("derive mode needs an all-sources sweep (strong scaling)")
    if args.mode != "batch" and wderive_ok:
        if args.wcover == "spf":
            leaf = shard.leaf_set(csr["row_ptr"], csr["col"])
            try:
                eng.cover_prepare(leaf)
            except Exception as e:  # outside the cover kernel's limits: per-root cover runs
                log(f"[rank {rank}] cover SPF unavailable ({e}); cover roots on the batch path")
            else:
                return wcover_main(args, eng, csr, names, stream, desc, V, E, world, rank,
                                   dist_on, dev, backend, coll_dev, leaf)
        return wderive_main(args, eng, csr, names, stream, desc, V, E, world, rank, dist_on, dev,
                            backend, coll_dev, weighted)
    pool = perm if n_roots <= 0 else perm[: min(n_roots, V)]
    nbrs = shard.distinct_neighbors(csr["row_ptr"], csr["col"])
    key = shard.first_neighbor(csr["row_ptr"], csr["col"]) if args.root_order != "random" \
        else None
    weak = args.roots_per_gpu > 0
    caps = shard.neighbor_caps(nbrs)
    classes = shard.make_classes(pool, caps, args.roots_per_gpu if weak else pool.size, key,
                                 max_grouped_words=1 if args.root_order == "auto" else None)
    if args.class_only:
        classes = [c for c in classes if c.cap == args.class_only]
        if not classes:
            raise SystemExit(f"no class with neighbour capacity {args.class_only}")
    for c in classes:
        x = c.extra
        if weak:  # ranks' slices of one step must not overlap: <= m / world each
            x["n"] = min(c.per_step, max(1, c.roots.size // world))
        else:  # strong: this rank's contiguous slice of the class, every step
            lo, hi = shard.rank_slice(c.roots.size, world, rank)
            x["mine"] = c.roots[lo:hi]
            x["n"] = hi - lo
            x["slot"] = -(-c.roots.size // world)  # gather slot per rank (padded)
    classes = [c for c in classes if c.extra["n"] > 0]
    B = sum(c.extra["n"] for c in classes)
    for c in classes:
        n, x = c.extra["n"], c.extra
        x["max_nbrs"] = int(max(1, nbrs[c.roots].max()))  # engine hint: sizes bit-planes
        x["plan"] = eng.plan(c.nh_words, flags, n_roots=n, max_root_neighbors=x["max_nbrs"])
        x["d_all"] = torch.from_numpy(c.roots.astype(np.int32)).to(dev)
        x["roots"] = torch.from_numpy(x["mine"].astype(np.int32)).to(dev) if not weak else \
            torch.empty(n, dtype=torch.int32, device=dev)
        x["dist"] = torch.empty((n, V), dtype=torch.int32, device=dev)
        x["nh"] = None if args.no_nh else torch.empty((n, V, c.nh_words), dtype=torch.int32,
                                                      device=dev)
        x["dig"] = torch.zeros((x.get("slot", n), 3), dtype=torch.int64, device=dev)
        x["stream"] = torch.cuda.current_stream() if args.serial_streams else \
            torch.cuda.Stream(device=dev)
        x["ev"] = []
    main_s = torch.cuda.current_stream()
    order = sorted(classes, key=lambda c: -c.cap)  # longest runs first

    def launch(c, stream_):
        x = c.extra
        eng.run_dev(x["roots"].data_ptr(), x["n"], c.nh_words, flags=flags,
                    d_dist=x["dist"].data_ptr(),
                    d_nh=x["nh"].data_ptr() if x["nh"] is not None else 0,
                    d_digest=x["dig"].data_ptr(), stream=stream_.cuda_stream,
                    max_root_neighbors=x["max_nbrs"])

    if args.class_only:  # profiling mode: the class alone, back to back
        for _ in range(args.reps):
            launch(classes[0], main_s)
        eng.sync(main_s.cuda_stream)
        log(f"class-only W={args.class_only}: {args.reps} launches of "
            f"{classes[0].extra['n']} roots")
        return

    def step(i: int, timed: bool):
        ready = torch.cuda.Event()
        ready.record(main_s)  # the previous step's gathers are queued on main_s
        done = []
        for c in order:
            x, n = c.extra, c.extra["n"]
            cs = x["stream"]
            with torch.cuda.stream(cs):
                cs.wait_event(ready)
                if weak:  # cyclic sweep of the class, disjoint slices per rank
                    start = ((i * world + rank) * n) % c.roots.size
                    idx = (torch.arange(n, device=dev) + start) % c.roots.size
                    torch.index_select(x["d_all"], 0, idx, out=x["roots"])
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record(cs)
                launch(c, cs)
                ev[1].record(cs)
            done.append(ev[1])
            if timed:
                x["ev"].append(ev)
        for e in done:
            main_s.wait_event(e)
        if dist_on:
            for c in classes:
                c.extra["gathered"] = shard.gather_digests(c.extra["dig"])

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
        t = torch.tensor([dt], dtype=torch.float64, device=coll_dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t.item())

    # digests of the LAST timed step, by root id (rank 0 sees every rank's)
    step_digest = {}
    if not weak:
        for c in classes:
            x = c.extra
            if dist_on:
                g = x["gathered"].cpu().numpy().view(np.uint64).reshape(world, x["slot"], 3)
                for r in range(world):
                    lo, hi = shard.rank_slice(c.roots.size, world, r)
                    for j, root in enumerate(c.roots[lo:hi]):
                        step_digest[int(root)] = g[r, j]
            else:
                d = x["dig"].cpu().numpy().view(np.uint64)
                for j, root in enumerate(x["mine"]):
                    step_digest[int(root)] = d[j]

    roots_total = world * B * args.steps if weak else pool.size * args.steps

    # roofline. The classes overlap on their streams inside the timed steps,
    # so each class is then timed ALONE (not part of `value`): R launches on
    # one stream bracketed by HIP events on that stream. A class launch is a
    # sequence of kernels; profiles/<round>/ holds the single-stream rocprofv3
    # per-kernel summary of each class alone, whose per-class sums match.
    iso_s = torch.cuda.Stream(device=dev)
    for c in classes:
        x = c.extra
        ms = []
        with torch.cuda.stream(iso_s):
            for _ in range(args.iso_reps + 1):
                a_, b_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a_.record(iso_s)
                launch(c, iso_s)
                b_.record(iso_s)
                b_.synchronize()
                ms.append(a_.elapsed_time(b_))
        x["iso_ms"] = float(np.median(ms[1:])) if len(ms) > 1 else float(ms[0])
        x["ms"] = [a_.elapsed_time(b_) for a_, b_ in x["ev"]]
    eng.sync(iso_s.cuda_stream)

    def class_roofline(c):
        x, p = c.extra, c.extra["plan"]
        n = x["n"]
        comp = compulsory_bytes(V, E, c.nh_words, n, p["variant"], p["slices"], weighted)
        alg = n * bytes_per_root(V, E, c.nh_words)
        sec = x["iso_ms"] / 1e3
        tr = pmc_traffic(args.profile_dir, f"variant{p['variant']}_cap{c.cap}", n)
        return {"cap": c.cap, "nh_words": c.nh_words, "variant": p["variant"],
                "roots_per_launch": n,
                "isolated_launch_ms": round(x["iso_ms"], 3),
                "compulsory_bytes": comp, "achieved": round(comp / sec / 1e9, 1),
                "frac": round(comp / sec / 1e9 / HBM_PEAK_GBS, 4),
                "alg_equiv_GBs": round(alg / sec / 1e9, 1),
                "traffic": tr, "traffic_GBs": round(tr / sec / 1e9, 1) if tr else None,
                "traffic_over_compulsory": round(tr / comp, 2) if tr else None}

    rl = [class_roofline(c) for c in classes]
    dom = max(rl, key=lambda r: r["isolated_launch_ms"])
    kname = {5: "multi-source BFS class launch (variant 5: msbfs init + level/settle pairs "
                "+ rows kernels)",
             7: "wave-per-root Dial class launch (variant 7: wdial_kernel + row digest)"}
    roofline = {
        "bound": "hbm", "achieved": dom["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": dom["frac"], "traffic": dom["traffic"],
        "kernel": kname.get(dom["variant"], f"variant {dom['variant']} class launch") +
        f", neighbour capacity {dom['cap']} ({dom['nh_words']} next-hop words)",
        "roots_per_launch": dom["roots_per_launch"], "avg_launch_ms": dom["isolated_launch_ms"],
        "compulsory_bytes": dom["compulsory_bytes"], "alg_equiv_GBs": dom["alg_equiv_GBs"],
        "traffic_GBs": dom["traffic_GBs"],
        "traffic_over_compulsory": dom["traffic_over_compulsory"],
        "classes": rl,
        "note": "achieved = compulsory bytes of the dominant class launch (dist + next-hop rows "
                "written, 4V(1+W) per run, plus the CSR reads its traversals need at least once: "
                "variant 5 one neighbour-id + offset scan per 64-root pass; per-root kernels one "
                "scan per run) / its isolated launch time (HIP events on its stream, alone); "
                "alg_equiv_GBs = the SURVEY 8(d) per-root-scan model, which batched traversals "
                "beat (not a roofline fraction); traffic = measured HBM bytes per launch "
                "(rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, profiles/<round>/pmc_traffic.json)",
    }

    classes_cfg = [{"cap": c.cap, "nh_words": c.nh_words, "roots_this_rank": c.extra["n"],
                    **{kk: c.extra["plan"][kk] for kk in ("variant", "slices", "block")},
                    "avg_launch_ms": round(float(np.mean(c.extra["ms"])), 3),
                    "isolated_launch_ms": round(c.extra["iso_ms"], 3)} for c in classes]
    report(args, stream, names, pool, step_digest, dt, roots_total, E, desc, n_roots, V, world,
           rank, dist_on, backend, int(world * B if weak else pool.size), classes_cfg, roofline,
           "weak" if weak else "strong", "batch")
    if dist_on:
        torch.distributed.destroy_process_group()


def derive_main(args, eng, csr, names, stream, desc, V, E, world, rank, dist_on, dev, backend,
                coll_dev):
    """All-sources step in derive mode (spf_msbfs.hip "derive"). Phase 1:
    ospf_levels_dev over this rank's closure (its roots + their neighbours):
    dist rows + byte level rows, one distance-only traversal per 64 roots.
    Phase 2: ospf_nh_derive_dev per width class: next-hop rows + digests of
    this rank's roots from the level rows. Ranks own the racks + fabric
    switches of a block of pods and the spines of a block of planes (fabric
    names; other graphs: slices of each width class)."""
    rp, col = csr["row_ptr"], csr["col"]
    perm = np.random.default_rng(SEED).permutation(V).astype(np.uint32)
    key = shard.first_neighbor(rp, col)
    caps = shard.neighbor_caps(shard.distinct_neighbors(rp, col))
    all_caps = sorted(set(caps.tolist()))

    def part(r):
        if world == 1:
            return perm
        fp = shard.fabric_partition(names, world, r)
        if fp is not None:
            return fp
        cls = shard.make_classes(perm, caps, V, key)
        return np.concatenate([c.roots[slice(*shard.rank_slice(c.roots.size, world, r))]
                               for c in cls])

    parts = [part(r) for r in range(world)]
    lkey = shard.last_neighbor(rp, col)
    cls_all = [{cap: shard.locality_order(p[caps[p] == cap], lkey) for cap in all_caps}
               for p in parts]
    mine = parts[rank]
    clo = shard.locality_order(shard.closure(mine, rp, col), key)
    pos = np.full(V, 0xFFFFFFFF, np.uint32)
    pos[clo] = np.arange(clo.size, dtype=np.uint32)
    t0 = time.time()
    d_clo = torch.from_numpy(clo.view(np.int32)).to(dev)
    d_pos = torch.from_numpy(pos.view(np.int32)).to(dev)
    lev = torch.empty((clo.size, eng.lev_pitch), dtype=torch.uint8, device=dev)
    dist = torch.empty((clo.size, V), dtype=torch.int32, device=dev)
    ldg = torch.empty((clo.size, 3), dtype=torch.int64, device=dev)
    nbrs = shard.distinct_neighbors(rp, col)
    flags = N.OSPF_WANT_DIST | N.OSPF_WANT_NH | N.OSPF_WANT_DIGEST
    classes = []
    for cap in all_caps:
        roots = cls_all[rank][cap]
        W = max(1, cap // 32) if cap > 16 else 1
        slot = max(1, max(c[cap].size for c in cls_all))
        # every class derives from the level rows (lane-16 kernel up to 4
        # words, the word-per-lane kernel above); --wide batch runs the wider
        # ones (spines) on the bit-plane batch path instead, on their own
        # stream, concurrently with phase 1 (they need no level rows)
        kind = "derive" if W <= 4 or args.wide == "derive" else "batch"
        c = dict(cap=cap, W=W, roots=roots, n=int(roots.size), kind=kind,
                 d=torch.from_numpy(roots.view(np.int32)).to(dev),
                 nh=torch.empty((max(1, roots.size), V, W), dtype=torch.int32, device=dev),
                 dig=torch.zeros((slot, 3), dtype=torch.int64, device=dev),
                 stream=torch.cuda.Stream(device=dev), ms=[])
        if kind == "batch" and roots.size:
            c["max_nbrs"] = int(max(1, nbrs[roots].max()))
            c["plan"] = eng.plan(W, flags, n_roots=int(roots.size),
                                 max_root_neighbors=c["max_nbrs"])
            c["dist"] = torch.empty((roots.size, V), dtype=torch.int32, device=dev)
        classes.append(c)
    log(f"[rank {rank}] derive: {mine.size} roots, closure {clo.size}, buffers "
        f"{(lev.numel() + dist.numel() * 4 + sum(c['nh'].numel() * 4 for c in classes)) / 2**30:.1f}"
        f" GiB in {time.time() - t0:.1f}s")
    main_s = torch.cuda.current_stream()

    def phase1(s_):
        eng.levels_dev(d_clo.data_ptr(), clo.size, lev.data_ptr(), d_dist=dist.data_ptr(),
                       d_lev_digest=ldg.data_ptr(), stream=s_.cuda_stream)

    def phase2(c, s_):
        if c["n"] and c["kind"] == "batch":
            eng.run_dev(c["d"].data_ptr(), c["n"], c["W"], flags=flags,
                        d_dist=c["dist"].data_ptr(), d_nh=c["nh"].data_ptr(),
                        d_digest=c["dig"].data_ptr(), stream=s_.cuda_stream,
                        max_root_neighbors=c["max_nbrs"])
        elif c["n"]:
            eng.nh_derive_dev(c["d"].data_ptr(), c["n"], c["W"], lev.data_ptr(), d_pos.data_ptr(),
                              c["nh"].data_ptr(), d_lev_digest=ldg.data_ptr(),
                              d_digest=c["dig"].data_ptr(), max_root_neighbors=c["cap"],
                              stream=s_.cuda_stream)

    p1_ms = []

    def launches(timed, base, tm=True):
        """One step's launches, rooted at stream `base` (tm: timing events)."""
        ev = (lambda: torch.cuda.Event(enable_timing=True)) if tm else torch.cuda.Event
        a_, b_ = ev(), ev()
        a_.record(base)
        done = []
        for c in classes:  # batch classes start with the step (no level rows needed)
            if c["kind"] == "batch":
                cs = c["stream"]
                cs.wait_event(a_)
                e0, e1 = ev(), ev()
                e0.record(cs)
                phase2(c, cs)
                e1.record(cs)
                done.append(e1)
                if timed:
                    c["ms"].append((e0, e1))
        phase1(base)
        b_.record(base)
        for c in sorted(classes, key=lambda c: -c["W"] * c["n"]):
            if c["kind"] == "batch":
                continue
            # OPENR_DERIVE_SERIAL=1: the classes one after another on the main
            # stream (experiment; default: each on its own stream)
            cs = base if os.environ.get("OPENR_DERIVE_SERIAL") == "1" else c["stream"]
            cs.wait_event(b_)
            e0, e1 = ev(), ev()
            e0.record(cs)
            phase2(c, cs)
            e1.record(cs)
            done.append(e1)
            if timed:
                c["ms"].append((e0, e1))
        for e in done:
            base.wait_event(e)
        if timed:
            p1_ms.append((a_, b_))

    graph = None

    def step(timed):
        if graph is not None:
            graph.replay()
        else:
            launches(timed, main_s)
        if dist_on:
            for c in classes:
                c["gathered"] = shard.gather_digests(c["dig"])

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    eng.sync(main_s.cuda_stream)
    graph_note = "off"
    if args.graph != "off":
        # the whole step (levels rounds, memsets, the width classes on their
        # streams) as one HIP graph: small topologies are launch-bound
        try:
            # one eager step on the capture stream first: the engine's scratch
            # is per stream and must exist before capture (no allocation inside)
            cap_s = torch.cuda.Stream(device=dev)
            cap_s.wait_stream(main_s)
            with torch.cuda.stream(cap_s):
                launches(False, cap_s, tm=False)
            cap_s.synchronize()
            eng.sync(cap_s.cuda_stream)
            g_ = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g_, stream=cap_s):
                launches(False, cap_s, tm=False)
            torch.cuda.synchronize()
            graph = g_
            graph.replay()
            torch.cuda.synchronize()
            eng.sync(main_s.cuda_stream)
            graph_note = "on"
        except Exception as e:  # capture not supported here: eager launches
            graph = None
            graph_note = f"off (capture failed: {str(e)[:120]})"
            torch.cuda.synchronize()
            log(f"[rank {rank}] graph capture failed, eager launches: {e}")
    if dist_on:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize()
    if dist_on:
        torch.distributed.barrier()
    dt = time.perf_counter() - t_start
    eng.sync(main_s.cuda_stream)
    if dist_on:
        t = torch.tensor([dt], dtype=torch.float64, device=coll_dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t.item())

    # digests of the last timed step by root id (rank 0 sees every rank's)
    step_digest = {}
    for c in classes:
        if dist_on:
            g = c["gathered"].cpu().numpy().view(np.uint64).reshape(world, -1, 3)
            for r in range(world):
                for j, root in enumerate(cls_all[r][c["cap"]]):
                    step_digest[int(root)] = g[r, j]
        else:
            d = c["dig"].cpu().numpy().view(np.uint64)
            for j, root in enumerate(c["roots"]):
                step_digest[int(root)] = d[j]

    # isolated launches (alone on one stream, HIP events on it): phase 1 and
    # each class's phase 2; the roofline of the dominant one
    iso_s = torch.cuda.Stream(device=dev)

    def iso(fn):
        ms = []
        with torch.cuda.stream(iso_s):
            for _ in range(args.iso_reps + 1):
                a_, b_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a_.record(iso_s)
                fn(iso_s)
                b_.record(iso_s)
                b_.synchronize()
                ms.append(a_.elapsed_time(b_))
        return float(np.median(ms[1:])) if len(ms) > 1 else float(ms[0])

    p1_iso = iso(phase1)
    for c in classes:
        c["iso_ms"] = iso(lambda s_, c=c: phase2(c, s_)) if c["n"] else 0.0
    eng.sync(iso_s.cuda_stream)
    scans = -(-clo.size // 64) * (4 * E + 4 * (V + 1))
    units = [{"launch": "levels", "kernel": "ospf_levels_dev (distance-only multi-source BFS: "
              "msbfs init + level/settle pairs + levrows)", "roots_per_launch": int(clo.size),
              "isolated_launch_ms": round(p1_iso, 3),
              "compulsory_bytes": int(clo.size) * 4 * V + scans,
              "traffic": pmc_traffic(args.profile_dir, "derive_levels", int(clo.size))}]
    for c in classes:
        if c["n"] and c["kind"] == "batch":
            p = c["plan"]
            units.append({"launch": f"batch_cap{c['cap']}",
                          "kernel": f"variant {p['variant']} class launch ({c['W']} next-hop "
                                    f"words: multi-source BFS with bit-planes)",
                          "cap": c["cap"], "nh_words": c["W"], "roots_per_launch": c["n"],
                          "isolated_launch_ms": round(c["iso_ms"], 3),
                          "compulsory_bytes": compulsory_bytes(V, E, c["W"], c["n"], p["variant"],
                                                               p["slices"], False),
                          "traffic": pmc_traffic(args.profile_dir,
                                                 f"variant{p['variant']}_cap{c['cap']}", c["n"])})
        elif c["n"]:
            units.append({"launch": f"derive_cap{c['cap']}",
                          "kernel": f"ospf_nh_derive_dev ("
                                    f"{'nh_derive16_kernel' if c['W'] <= 4 else 'nh_derive_wide_kernel'}"
                                    f", {c['W']} next-hop word(s))", "cap": c["cap"], "nh_words": c["W"],
                          "roots_per_launch": c["n"], "isolated_launch_ms": round(c["iso_ms"], 3),
                          "compulsory_bytes": c["n"] * 4 * V * c["W"],
                          "traffic": pmc_traffic(args.profile_dir, f"derive_cap{c['cap']}", c["n"])})
    for u in units:
        sec = u["isolated_launch_ms"] / 1e3
        u["achieved"] = round(u["compulsory_bytes"] / sec / 1e9, 1)
        u["frac"] = round(u["compulsory_bytes"] / sec / 1e9 / HBM_PEAK_GBS, 4)
        u["traffic_over_compulsory"] = (round(u["traffic"] / u["compulsory_bytes"], 2)
                                        if u["traffic"] else None)
    dom = max(units, key=lambda u: u["isolated_launch_ms"])
    step_comp = sum(c["n"] * 4 * V * (1 + c["W"]) for c in classes) + scans + sum(
        -(-c["n"] // 64) * c["plan"]["slices"] * (4 * E + 4 * (V + 1))
        for c in classes if c["kind"] == "batch" and c["n"])
    step_s = dt / args.steps
    roofline = {
        "bound": "hbm", "achieved": dom["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": dom["frac"], "traffic": dom["traffic"], "kernel": dom["kernel"],
        "roots_per_launch": dom["roots_per_launch"], "avg_launch_ms": dom["isolated_launch_ms"],
        "compulsory_bytes": dom["compulsory_bytes"],
        "traffic_over_compulsory": dom["traffic_over_compulsory"], "launches": units,
        "step_compulsory_bytes": step_comp,
        "step_frac": round(step_comp / step_s / 1e9 / HBM_PEAK_GBS, 4),
        "note": "achieved = compulsory bytes of the dominant launch / its isolated time (HIP "
                "events on its stream, alone): levels = dist rows written (4V per run) + one "
                "neighbour-id + offset scan per 64-root traversal; derive = next-hop rows "
                "written (4VW per run); the byte level rows are intermediate (traffic, not "
                "compulsory). step_frac = (dist + next-hop rows of every root + scans) / "
                "ms_per_step. traffic = measured HBM bytes per launch (rocprofv3 FETCH_SIZE x2 "
                "+ WRITE_SIZE, profiles/<round>/pmc_traffic.json)",
    }
    p1_avg = float(np.mean([a_.elapsed_time(b_) for a_, b_ in p1_ms])) if p1_ms else None
    classes_cfg = [{"launch": "levels", "roots_this_rank": int(clo.size),
                    "closure_over_roots": round(clo.size / max(1, mine.size), 4),
                    "avg_launch_ms": round(p1_avg, 3) if p1_avg is not None else None,
                    "isolated_launch_ms": round(p1_iso, 3), "hip_graph": graph_note}]
    for c in classes:
        classes_cfg.append({"cap": c["cap"], "nh_words": c["W"], "roots_this_rank": c["n"],
                            "path": c["kind"],
                            "avg_launch_ms": round(float(np.mean(
                                [a_.elapsed_time(b_) for a_, b_ in c["ms"]])), 3) if c["ms"] else None,
                            "isolated_launch_ms": round(c["iso_ms"], 3)})
    report(args, stream, names, perm, step_digest, dt, V * args.steps, E, desc, 0, V, world, rank,
           dist_on, backend, V, classes_cfg, roofline, "strong", "derive")
    if dist_on:
        torch.distributed.destroy_process_group()


def wcover_main(args, eng, csr, names, stream, desc, V, E, world, rank, dist_on, dev, backend,
                coll_dev, leaf):
    """All-sources step on a weighted graph, cover SPF form. (A) dist rows of
    the cover (nodes outside the independent leaf set: the fabric and spine
    switches) by the contracted-graph SPF (spf_cover.hip); (B) the leaves'
    dist + next-hop rows from those rows (ospf_wderive_dev); (C) the next hops
    of cover roots with <= 128 neighbours from their own and their
    neighbours' rows (ospf_wderive_wide_dev). Wider cover roots (spines) run
    the per-root batch kernel on their own stream from the step's start. A
    rank owns a pod / plane block (fabric) or class slices, and computes the
    rows its own roots' derivations read."""
    rp, col = csr["row_ptr"], csr["col"]
    perm = np.random.default_rng(SEED).permutation(V).astype(np.uint32)
    key = shard.first_neighbor(rp, col)
    nbrs = shard.distinct_neighbors(rp, col)
    caps = shard.neighbor_caps(nbrs)
    words = np.maximum(1, (nbrs + 31) // 32)
    # cover next hops: roots sharing their largest neighbours side by side (the
    # fabric switches of a pod share its racks' rows); OPENR_WCOVER_KEY=first
    # groups them by their smallest neighbour instead
    ckey = key if os.environ.get("OPENR_WCOVER_KEY") == "first" else shard.last_neighbor(rp, col)

    def part(r):
        if world == 1:
            return perm
        fp = shard.fabric_partition(names, world, r)
        if fp is not None:
            return fp
        cls = shard.make_classes(perm, caps, V, key)
        return np.concatenate([c.roots[slice(*shard.rank_slice(c.roots.size, world, r))]
                               for c in cls])

    def plan(p):
        p = np.asarray(p, np.uint32)
        own_l = shard.locality_order(p[leaf[p]], key)
        own_c = p[~leaf[p]]
        c_der = own_c[(nbrs[own_c] <= 2048)]         # (C): next hops derived
        c_wide = own_c[(nbrs[own_c] > 2048)]         # per-root batch kernel
        nb_c = shard.closure(c_der, rp, col)
        need_l = np.union1d(own_l, nb_c[leaf[nb_c]]).astype(np.uint32)
        need_l = shard.locality_order(need_l, key)
        cl = shard.closure(need_l, rp, col)
        cover_a = np.union1d(np.union1d(own_c, cl[~leaf[cl]]), nb_c[~leaf[nb_c]]).astype(np.uint32)
        return dict(own_l=own_l, c_der=c_der, c_wide=c_wide, need_l=need_l, cover_a=cover_a)

    parts = [part(r) for r in range(world)]
    plans = [plan(p) for p in parts]
    P = plans[rank]
    cover_a, need_l = P["cover_a"], P["need_l"]
    nA, nL = int(cover_a.size), int(need_l.size)
    pos = np.full(V, 0xFFFFFFFF, np.uint32)
    pos[cover_a] = np.arange(nA, dtype=np.uint32)
    pos[need_l] = nA + np.arange(nL, dtype=np.uint32)
    t0 = time.time()
    slab = torch.empty((max(1, nA + nL), V), dtype=torch.int32, device=dev)
    d_pos = torch.from_numpy(pos.view(np.int32)).to(dev)
    d_a = torch.from_numpy(cover_a.view(np.int32)).to(dev)
    d_l = torch.from_numpy(need_l.view(np.int32)).to(dev)
    lnh = torch.empty((max(1, nL), V), dtype=torch.int32, device=dev)
    ldg = torch.zeros((max(1, nL), 3), dtype=torch.int64, device=dev)
    kmax = int(nbrs[need_l].max()) if nL else 0
    flags = N.OSPF_WANT_DIST | N.OSPF_WANT_NH | N.OSPF_WANT_DIGEST
    cls = []  # (C) classes by next-hop words, and the wide batch class
    for W in sorted(set(words[P["c_der"]].tolist())):
        roots = shard.locality_order(P["c_der"][words[P["c_der"]] == W], ckey)
        cls.append(dict(kind="derive", W=W, roots=roots, n=int(roots.size),
                        d=torch.from_numpy(roots.view(np.int32)).to(dev),
                        nh=torch.empty((roots.size, V, W), dtype=torch.int32, device=dev),
                        dig=torch.zeros((roots.size, 3), dtype=torch.int64, device=dev), ms=[],
                        side=torch.cuda.Stream(device=dev)))
    if P["c_wide"].size:
        roots = shard.locality_order(P["c_wide"], key)
        W = int(words[roots].max())
        mx = int(nbrs[roots].max())
        cls.append(dict(kind="batch", W=W, roots=roots, n=int(roots.size), max_nbrs=mx,
                        plan=eng.plan(W, flags, n_roots=int(roots.size), max_root_neighbors=mx),
                        d=torch.from_numpy(roots.view(np.int32)).to(dev),
                        nh=torch.empty((roots.size, V, W), dtype=torch.int32, device=dev),
                        dist=torch.empty((roots.size, V), dtype=torch.int32, device=dev),
                        dig=torch.zeros((roots.size, 3), dtype=torch.int64, device=dev),
                        stream=torch.cuda.Stream(device=dev), ms=[]))
    log(f"[rank {rank}] wcover: {parts[rank].size} roots: cover SPF {nA}, leaves {nL} "
        f"(<= {kmax} neighbours), cover next hops {[(c['kind'], c['W'], c['n']) for c in cls]}, "
        f"buffers {(slab.numel() + lnh.numel() + sum(c['nh'].numel() for c in cls)) * 4 / 2**30:.1f}"
        f" GiB in {time.time() - t0:.1f}s")
    main_s = torch.cuda.current_stream()

    def stage_a(s_):
        eng.cover_dist_dev(d_a.data_ptr(), nA, slab.data_ptr(), stream=s_.cuda_stream)

    def stage_b(s_):
        if nL:
            eng.wderive_dev(d_l.data_ptr(), nL, slab.data_ptr(), d_pos.data_ptr(),
                            slab[nA].data_ptr(), d_nh=lnh.data_ptr(), d_digest=ldg.data_ptr(),
                            max_root_neighbors=kmax, stream=s_.cuda_stream)

    def stage_c(c, s_):
        if c["kind"] == "derive":
            eng.wderive_wide_dev(c["d"].data_ptr(), c["n"], c["W"], slab.data_ptr(),
                                 d_pos.data_ptr(), c["nh"].data_ptr(),
                                 d_digest=c["dig"].data_ptr(), stream=s_.cuda_stream)
        else:
            eng.run_dev(c["d"].data_ptr(), c["n"], c["W"], flags=flags,
                        d_dist=c["dist"].data_ptr(), d_nh=c["nh"].data_ptr(),
                        d_digest=c["dig"].data_ptr(), stream=s_.cuda_stream,
                        max_root_neighbors=c["max_nbrs"])

    # owned roots' digests, gathered in a padded slot per rank
    def owned_order(p, pl):
        own = np.zeros(V, bool)
        own[p] = True
        lo = pl["need_l"][own[pl["need_l"]]]
        co = [shard.locality_order(pl["c_der"][words[pl["c_der"]] == W], ckey)
              for W in sorted(set(words[pl["c_der"]].tolist()))]
        if pl["c_wide"].size:
            co.append(shard.locality_order(pl["c_wide"], key))
        return np.concatenate([lo] + co) if (lo.size or co) else lo

    owned = [owned_order(p, pl) for p, pl in zip(parts, plans)]
    slot = max(o.size for o in owned)
    gbuf = torch.zeros((slot, 3), dtype=torch.int64, device=dev)
    own_l_idx = torch.from_numpy(np.nonzero(np.isin(need_l, parts[rank]))[0].astype(np.int64)).to(dev)
    stage_ms, gathered = {"A": [], "B": [], "C": []}, {}

    def step(timed):
        a0 = torch.cuda.Event(enable_timing=True)
        a0.record(main_s)
        done = []
        for c in cls:  # wide cover roots: their own batch, from the start
            if c["kind"] == "batch":
                c["stream"].wait_event(a0)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(c["stream"])
                stage_c(c, c["stream"])
                e1.record(c["stream"])
                done.append(e1)
                if timed:
                    c["ms"].append((e0, e1))
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        stage_a(main_s)
        ev[1].record(main_s)
        # wide cover roots (spines) need only the cover rows: their derivation
        # runs beside the leaves' and the narrow cover roots'
        for c in cls:
            if c["kind"] == "derive" and c["W"] > 4:
                c["side"].wait_event(ev[1])
                stage_c(c, c["side"])
                e1 = torch.cuda.Event()
                e1.record(c["side"])
                done.append(e1)
        stage_b(main_s)
        ev[2].record(main_s)
        for c in cls:
            if c["kind"] == "derive" and c["W"] <= 4:
                stage_c(c, main_s)
        ev[3].record(main_s)
        for e in done:
            main_s.wait_event(e)
        if timed:
            stage_ms["A"].append((a0, ev[1]))
            stage_ms["B"].append((ev[1], ev[2]))
            stage_ms["C"].append((ev[2], ev[3]))
        if dist_on:
            parts_ = [torch.index_select(ldg, 0, own_l_idx)] + [c["dig"] for c in cls]
            cat = torch.cat(parts_)
            gbuf[: cat.shape[0]].copy_(cat)
            gathered["g"] = shard.gather_digests(gbuf)

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    eng.sync(main_s.cuda_stream)
    if dist_on:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize()
    if dist_on:
        torch.distributed.barrier()
    dt = time.perf_counter() - t_start
    eng.sync(main_s.cuda_stream)
    if dist_on:
        t = torch.tensor([dt], dtype=torch.float64, device=coll_dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t.item())

    step_digest = {}
    if dist_on:
        g = gathered["g"].cpu().numpy().view(np.uint64).reshape(world, slot, 3)
        for r, o in enumerate(owned):
            for j, root in enumerate(o):
                step_digest[int(root)] = g[r, j]
    else:
        ld = ldg.cpu().numpy().view(np.uint64)
        for j, root in enumerate(need_l):
            step_digest[int(root)] = ld[j]
        for c in cls:
            d = c["dig"].cpu().numpy().view(np.uint64)
            for j, root in enumerate(c["roots"]):
                step_digest[int(root)] = d[j]

    iso_s = torch.cuda.Stream(device=dev)

    def iso(fn):
        ms = []
        with torch.cuda.stream(iso_s):
            for _ in range(args.iso_reps + 1):
                a_, b_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a_.record(iso_s)
                fn(iso_s)
                b_.record(iso_s)
                b_.synchronize()
                ms.append(a_.elapsed_time(b_))
        return float(np.median(ms[1:])) if len(ms) > 1 else float(ms[0])

    scan_c = 8 * E + 4 * (V + 1)  # one weighted CSR scan (neighbour + metric words)
    units = [{"launch": "cover_spf", "kernel": "ospf_cover_dist_dev (cover_spf_kernel: "
              "contracted-graph Dial, LDS-resident distances)", "roots_per_launch": nA,
              "isolated_launch_ms": round(iso(stage_a), 3),
              "compulsory_bytes": nA * 4 * V + scan_c,
              "traffic": pmc_traffic(args.profile_dir, "cover_spf", nA)}]
    if nL:
        units.append({"launch": "wderive", "kernel": "ospf_wderive_dev (wderive_kernel: leaf "
                      "rows from the cover rows)", "roots_per_launch": nL,
                      "isolated_launch_ms": round(iso(stage_b), 3),
                      "compulsory_bytes": nL * 8 * V + int(np.setdiff1d(shard.closure(
                          need_l, rp, col), need_l).size) * 4 * V,
                      "traffic": pmc_traffic(args.profile_dir, "wderive", nL)})
    for c in cls:
        c["iso_ms"] = iso(lambda s_, c=c: stage_c(c, s_))
        if c["kind"] == "derive":
            units.append({"launch": f"wderive_wide_w{c['W']}", "kernel": f"ospf_wderive_wide_dev "
                          f"(wderive_wide_kernel<{c['W']}>)", "roots_per_launch": c["n"],
                          "isolated_launch_ms": round(c["iso_ms"], 3),
                          "compulsory_bytes": c["n"] * 4 * V * c["W"],
                          "traffic": pmc_traffic(args.profile_dir, f"wderive_wide_w{c['W']}",
                                                 c["n"])})
        else:
            p = c["plan"]
            units.append({"launch": f"cover_batch_w{c['W']}",
                          "kernel": f"variant {p['variant']} class launch ({c['W']} next-hop words)",
                          "roots_per_launch": c["n"], "isolated_launch_ms": round(c["iso_ms"], 3),
                          "compulsory_bytes": compulsory_bytes(V, E, c["W"], c["n"], p["variant"],
                                                               p["slices"], True),
                          "traffic": pmc_traffic(args.profile_dir,
                                                 f"variant{p['variant']}_cap{c['W'] * 32}", c["n"])})
    eng.sync(iso_s.cuda_stream)
    for u in units:
        sec = u["isolated_launch_ms"] / 1e3
        u["achieved"] = round(u["compulsory_bytes"] / sec / 1e9, 1)
        u["frac"] = round(u["compulsory_bytes"] / sec / 1e9 / HBM_PEAK_GBS, 4)
        u["traffic_over_compulsory"] = (round(u["traffic"] / u["compulsory_bytes"], 2)
                                        if u["traffic"] else None)
    dom = max(units, key=lambda u: u["isolated_launch_ms"])
    step_comp = sum(u["compulsory_bytes"] for u in units)
    step_s = dt / args.steps
    roofline = {
        "bound": "hbm", "achieved": dom["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": dom["frac"], "traffic": dom["traffic"], "kernel": dom["kernel"],
        "roots_per_launch": dom["roots_per_launch"], "avg_launch_ms": dom["isolated_launch_ms"],
        "compulsory_bytes": dom["compulsory_bytes"],
        "traffic_over_compulsory": dom["traffic_over_compulsory"], "launches": units,
        "step_compulsory_bytes": step_comp,
        "step_frac": round(step_comp / step_s / 1e9 / HBM_PEAK_GBS, 4),
        "note": "achieved = compulsory bytes of the dominant launch / its isolated time: "
                "cover_spf = dist rows written + one weighted CSR scan; wderive = leaf dist + "
                "next-hop rows + the cover rows read once; wderive_wide = next-hop rows; "
                "cover_batch = rows + one weighted CSR scan per run",
    }
    cfg = [{"launch": k, "avg_launch_ms": round(float(np.mean([a_.elapsed_time(b_) for a_, b_ in v])), 3)}
           for k, v in stage_ms.items() if v]
    cfg += [{"launch": f"cover_batch_w{c['W']}", "roots_this_rank": c["n"],
             "avg_launch_ms": round(float(np.mean([a_.elapsed_time(b_) for a_, b_ in c["ms"]])), 3)}
            for c in cls if c["kind"] == "batch"]
    report(args, stream, names, perm, step_digest, dt, V * args.steps, E, desc, 0, V, world, rank,
           dist_on, backend, V, cfg, roofline, "strong", "wcover")
    if dist_on:
        torch.distributed.destroy_process_group()


def wderive_main(args, eng, csr, names, stream, desc, V, E, world, rank, dist_on, dev, backend,
                 coll_dev, weighted):
    """All-sources step on a weighted graph (or any graph outside derive
    mode's unit-metric contract). Cover roots (a vertex cover S: on the
    fabric the fabric and spine switches) run the per-root SPF kernel chosen
    by the engine (variant 7 here), one launch per width class on its own
    stream, their dist rows into one slab; then the leaf roots (the
    independent set I = V \\ S: the racks) are derived from those rows by
    ospf_wderive_dev (spf_wderive.hip). A rank owns a pod / plane block
    (fabric) or class slices, and runs the cover rows its leaves need."""
    rp, col = csr["row_ptr"], csr["col"]
    perm = np.random.default_rng(SEED).permutation(V).astype(np.uint32)
    key = shard.first_neighbor(rp, col)
    nbrs = shard.distinct_neighbors(rp, col)
    caps = shard.neighbor_caps(nbrs)
    leaf = shard.leaf_set(rp, col)

    def part(r):
        if world == 1:
            return perm
        fp = shard.fabric_partition(names, world, r)
        if fp is not None:
            return fp
        cls = shard.make_classes(perm, caps, V, key)
        return np.concatenate([c.roots[slice(*shard.rank_slice(c.roots.size, world, r))]
                               for c in cls])

    parts = [part(r) for r in range(world)]
    plans = [shard.wderive_plan(p, leaf, rp, col) for p in parts]
    cover, lr = plans[rank]
    lr = shard.locality_order(lr, key)  # racks of a pod adjacent: one run per pod
    flags = N.OSPF_WANT_DIST | N.OSPF_WANT_NH | N.OSPF_WANT_DIGEST
    t0 = time.time()
    classes, off = [], 0
    for cap in sorted(set(caps[cover].tolist())):
        roots = shard.locality_order(cover[caps[cover] == cap], key)
        W = max(1, cap // 32) if cap > 16 else 1
        mx = int(max(1, nbrs[roots].max()))
        classes.append(dict(cap=cap, W=W, roots=roots, n=int(roots.size), off=off,
                            d=torch.from_numpy(roots.view(np.int32)).to(dev),
                            nh=torch.empty((roots.size, V, W), dtype=torch.int32, device=dev),
                            max_nbrs=mx,
                            plan=eng.plan(W, flags, n_roots=int(roots.size),
                                          max_root_neighbors=mx),
                            stream=torch.cuda.Stream(device=dev), ms=[]))
        off += roots.size
    corder = np.concatenate([c["roots"] for c in classes]) if classes else \
        np.zeros(0, np.uint32)
    pos = np.full(V, 0xFFFFFFFF, np.uint32)
    pos[corder] = np.arange(corder.size, dtype=np.uint32)
    cdist = torch.empty((max(1, corder.size), V), dtype=torch.int32, device=dev)
    d_pos = torch.from_numpy(pos.view(np.int32)).to(dev)
    nl = int(lr.size)
    kmax = int(nbrs[lr].max()) if nl else 0
    d_lr = torch.from_numpy(lr.view(np.int32)).to(dev)
    ldist = torch.empty((max(1, nl), V), dtype=torch.int32, device=dev)
    lnh = torch.empty((max(1, nl), V), dtype=torch.int32, device=dev)
    dig = torch.zeros((corder.size + nl, 3), dtype=torch.int64, device=dev)
    log(f"[rank {rank}] wderive: {parts[rank].size} roots = {nl} leaves (<= {kmax} "
        f"neighbours) + cover {corder.size} ({[(c['cap'], c['n'], c['plan']['variant']) for c in classes]}), "
        f"buffers {(cdist.numel() + ldist.numel() + lnh.numel() + sum(c['nh'].numel() for c in classes)) * 4 / 2**30:.1f}"
        f" GiB in {time.time() - t0:.1f}s")
    main_s = torch.cuda.current_stream()

    def cover_launch(c, s_):
        eng.run_dev(c["d"].data_ptr(), c["n"], c["W"], flags=flags,
                    d_dist=cdist[c["off"]].data_ptr(), d_nh=c["nh"].data_ptr(),
                    d_digest=dig[c["off"]].data_ptr(), stream=s_.cuda_stream,
                    max_root_neighbors=c["max_nbrs"])

    def leaf_launch(s_):
        if nl:
            eng.wderive_dev(d_lr.data_ptr(), nl, cdist.data_ptr(), d_pos.data_ptr(),
                            ldist.data_ptr(), d_nh=lnh.data_ptr(),
                            d_digest=dig[corder.size].data_ptr(), max_root_neighbors=kmax,
                            stream=s_.cuda_stream)

    # owned roots' digest rows (the cover rows a rank adds for its leaves are
    # not its roots), gathered in a padded slot per rank
    def owned_rows(p, cv, lv):
        own = np.zeros(V, bool)
        own[p] = True
        co = np.concatenate([shard.locality_order(cv[caps[cv] == cap], key)
                             for cap in sorted(set(caps[cv].tolist()))]) if cv.size else cv
        return co[own[co]], shard.locality_order(lv, key)

    owned = [owned_rows(p, *pl) for p, pl in zip(parts, plans)]
    slot = max(a.size + b.size for a, b in owned)
    own_c, _ = owned[rank]
    idx = np.concatenate([pos[own_c], corder.size + np.arange(nl)]).astype(np.int64)
    d_idx = torch.from_numpy(idx).to(dev)
    gbuf = torch.zeros((slot, 3), dtype=torch.int64, device=dev)
    leaf_ms, gathered = [], {}

    def step(timed):
        a_ = torch.cuda.Event(enable_timing=True)
        a_.record(main_s)
        done = []
        for c in classes:
            cs = c["stream"]
            cs.wait_event(a_)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(cs)
            cover_launch(c, cs)
            e1.record(cs)
            done.append(e1)
            if timed:
                c["ms"].append((e0, e1))
        for e in done:
            main_s.wait_event(e)
        l0, l1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        l0.record(main_s)
        leaf_launch(main_s)
        l1.record(main_s)
        if timed:
            leaf_ms.append((l0, l1))
        if dist_on:
            torch.index_select(dig, 0, d_idx, out=gbuf[: idx.size])
            gathered["g"] = shard.gather_digests(gbuf)

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    eng.sync(main_s.cuda_stream)
    if dist_on:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize()
    if dist_on:
        torch.distributed.barrier()
    dt = time.perf_counter() - t_start
    eng.sync(main_s.cuda_stream)
    if dist_on:
        t = torch.tensor([dt], dtype=torch.float64, device=coll_dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t.item())

    step_digest = {}
    if dist_on:
        g = gathered["g"].cpu().numpy().view(np.uint64).reshape(world, slot, 3)
        for r, (a, b) in enumerate(owned):
            for j, root in enumerate(np.concatenate([a, b])):
                step_digest[int(root)] = g[r, j]
    else:
        d = dig.cpu().numpy().view(np.uint64)
        for j, root in enumerate(np.concatenate([corder, lr])):
            step_digest[int(root)] = d[j]

    iso_s = torch.cuda.Stream(device=dev)

    def iso(fn):
        ms = []
        with torch.cuda.stream(iso_s):
            for _ in range(args.iso_reps + 1):
                a_, b_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a_.record(iso_s)
                fn(iso_s)
                b_.record(iso_s)
                b_.synchronize()
                ms.append(a_.elapsed_time(b_))
        return float(np.median(ms[1:])) if len(ms) > 1 else float(ms[0])

    units = []
    for c in classes:
        c["iso_ms"] = iso(lambda s_, c=c: cover_launch(c, s_))
        p = c["plan"]
        units.append({"launch": f"cover_cap{c['cap']}",
                      "kernel": f"variant {p['variant']} class launch ({c['W']} next-hop words)",
                      "cap": c["cap"], "nh_words": c["W"], "roots_per_launch": c["n"],
                      "isolated_launch_ms": round(c["iso_ms"], 3),
                      "compulsory_bytes": compulsory_bytes(V, E, c["W"], c["n"], p["variant"],
                                                           p["slices"], weighted),
                      "traffic": pmc_traffic(args.profile_dir,
                                             f"variant{p['variant']}_cap{c['cap']}", c["n"])})
    if nl:
        l_iso = iso(leaf_launch)
        n_src = int(np.setdiff1d(shard.closure(lr, rp, col), lr).size)  # cover rows read
        units.append({"launch": "wderive", "kernel": "ospf_wderive_dev (wderive_kernel: leaf "
                      "rows from neighbours' dist rows)", "roots_per_launch": nl,
                      "isolated_launch_ms": round(l_iso, 3),
                      "compulsory_bytes": nl * 8 * V + n_src * 4 * V,
                      "traffic": pmc_traffic(args.profile_dir, "wderive", nl)})
    eng.sync(iso_s.cuda_stream)
    for u in units:
        sec = u["isolated_launch_ms"] / 1e3
        u["achieved"] = round(u["compulsory_bytes"] / sec / 1e9, 1)
        u["frac"] = round(u["compulsory_bytes"] / sec / 1e9 / HBM_PEAK_GBS, 4)
        u["traffic_over_compulsory"] = (round(u["traffic"] / u["compulsory_bytes"], 2)
                                        if u["traffic"] else None)
    dom = max(units, key=lambda u: u["isolated_launch_ms"])
    step_comp = sum(u["compulsory_bytes"] for u in units)
    step_s = dt / args.steps
    roofline = {
        "bound": "hbm", "achieved": dom["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": dom["frac"], "traffic": dom["traffic"], "kernel": dom["kernel"],
        "roots_per_launch": dom["roots_per_launch"], "avg_launch_ms": dom["isolated_launch_ms"],
        "compulsory_bytes": dom["compulsory_bytes"],
        "traffic_over_compulsory": dom["traffic_over_compulsory"], "launches": units,
        "step_compulsory_bytes": step_comp,
        "step_frac": round(step_comp / step_s / 1e9 / HBM_PEAK_GBS, 4),
        "note": "achieved = compulsory bytes of the dominant launch / its isolated time: cover "
                "classes = dist + next-hop rows written + one weighted CSR scan per run; "
                "wderive = leaf dist + next-hop rows written + the cover rows read once",
    }
    classes_cfg = [{"cap": c["cap"], "nh_words": c["W"], "roots_this_rank": c["n"],
                    "path": f"cover (variant {c['plan']['variant']})",
                    "avg_launch_ms": round(float(np.mean([a_.elapsed_time(b_) for a_, b_ in c["ms"]])), 3),
                    "isolated_launch_ms": round(c["iso_ms"], 3)} for c in classes]
    if nl:
        classes_cfg.append({"launch": "wderive", "roots_this_rank": nl, "max_neighbours": kmax,
                            "avg_launch_ms": round(float(np.mean(
                                [a_.elapsed_time(b_) for a_, b_ in leaf_ms])), 3),
                            "isolated_launch_ms": round(l_iso, 3)})
    report(args, stream, names, perm, step_digest, dt, V * args.steps, E, desc, 0, V, world, rank,
           dist_on, backend, V, classes_cfg, roofline, "strong", "wderive")
    if dist_on:
        torch.distributed.destroy_process_group()


def report(args, stream, names, pool, step_digest, dt, roots_total, E, desc, n_roots, V, world,
           rank, dist_on, backend, roots_per_step, classes_cfg, roofline, scaling, mode):
    """CPU baseline + parity of the timed step's digests (rank 0) and the one
    JSON line."""
    spf_s = roots_total / dt
    gteps = roots_total * E / dt / 1e9
    cpu = parity = None
    if rank == 0 and world == 1 and not args.no_cpu:
        from oracle import Oracle  # CPU baseline leg only (the restatements under oracle/)
        threads = args.cpu_threads or host_threads()
        k = args.cpu_sample if args.cpu_sample >= 0 else (16 if args.topology == "mesh1m" else 256)
        sample_ids = [int(r) for r in pool[:k]]
        sample = [names[i] for i in sample_ids]
        o = Oracle(stream)
        # reference-shaped restatement (string keys, hash sets, heap + make_heap
        # per strict improvement): quadratic on weighted fabrics (~10 min per
        # F100k root), so there the CSR-Dijkstra restatement is the baseline
        ref_ok = args.topology != "fabric100k-w"
        mesh = args.topology == "mesh1m"
        csr_k = 64 if mesh else max(k, 256)  # ~2 s per M1M root on one core
        csr_ids = [int(r) for r in pool[:csr_k]]
        t1 = time.perf_counter()
        fd = o.fast_digests([names[i] for i in csr_ids], threads=threads)
        ct_fast = time.perf_counter() - t1
        csr_line = {"value": round(len(csr_ids) / ct_fast, 3), "unit": "SPF/s",
                    "cores": threads, "kind": "port",
                    "sample": f"{len(csr_ids)} roots (permutation seed 0x5eed), CSR-Dijkstra "
                              f"restatement (oracle/, integer ids, binary heap), {threads} "
                              f"threads, {ct_fast:.2f}s"}
        checks = dict(zip(csr_ids, fd))
        if ref_ok:
            n1 = 1 if mesh else 2
            t1 = time.perf_counter()
            one = o.digests(sample[:n1], threads=1)
            st_s = (time.perf_counter() - t1) / n1
            t1 = time.perf_counter()
            cd = o.digests(sample, threads=threads)
            ct = time.perf_counter() - t1
            assert np.array_equal(one, cd[:n1])
            cpu = {"value": round(len(sample) / ct, 4), "unit": "SPF/s", "cores": threads,
                   "kind": "port",
                   "sample": f"{len(sample)} roots (permutation seed 0x5eed) of the same "
                             f"topology, reference-shaped runSpf restatement (oracle/: string "
                             f"keys, hash sets, heap + make_heap), {threads} threads, {ct:.2f}s",
                   "cpu_model": cpu_model(), "single_thread_s_per_root": round(st_s, 4),
                   "csr_dijkstra": csr_line}
            checks.update(zip(sample_ids, cd))
        else:
            cpu = dict(csr_line, cpu_model=cpu_model(),
                       reference_shaped="not run: its make_heap per strict improvement "
                                        "(LinkState.cpp:893) takes ~10 min per root here")
        if step_digest:
            parity = {"roots": len(checks),
                      "equal": bool(all(np.array_equal(step_digest[r], d)
                                        for r, d in checks.items())),
                      "source": "digests of the last timed step vs the CPU restatement(s)"}

    if rank == 0 and dist_on and args.dist_parity > 0 and step_digest:
        from oracle import Oracle  # checker only, after the timed region
        ids = [int(r) for r in pool[: args.dist_parity]]
        want = Oracle(stream).fast_digests([names[i] for i in ids], threads=host_threads())
        parity = {"roots": len(ids),
                  "equal": bool(all(np.array_equal(step_digest[r], w) for r, w in zip(ids, want))),
                  "source": "all-gathered digests of the last timed step (every rank's shard) "
                            "vs the CSR-Dijkstra restatement"}

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(spf_s, 2), "unit": "SPF/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": scaling, "vs_baseline": None, "dtype": "u32",
            "data": "synthetic", "gteps": round(gteps, 3),
            "config": {
                "workload": desc + (" all-sources" if n_roots <= 0 else
                                    f" {pool.size} sampled roots") +
                " SPF + ECMP next-hop bitsets (dist + next-hop rows written to HBM, per-root "
                "digests)",
                "n_nodes": V, "n_directed_edges": E, "mode": mode,
                "roots_per_step": roots_per_step,
                "root_classes": classes_cfg,
                "parallelism": f"root-sharded x{world}" +
                               (f", all_gather of 24-B digests ({'RCCL' if backend == 'nccl' else backend})"
                                if dist_on else "")},
            "roofline": roofline, "cpu_baseline": cpu, "parity_vs_cpu_sample": parity,
        }
        if dist_on:
            line["gathered_roots"] = len(step_digest)
            line["dist_backend"] = backend
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
