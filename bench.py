#!/usr/bin/env python3
"""Benchmark: all-sources SPF + ECMP next hops on the 100k-node fabric.

BASELINE.json metric: "all-sources SPF/sec + GTEPS on 100k-node fabric
topology at 1/2/4/8 GPUs". A *step* = one all-sources sweep: every node of
the topology is the root of one SPF run (LinkState::runSpf,
openr/decision/LinkState.cpp:836-911) whose distance row and next-hop bitset
row are written to HBM, plus a 24-B digest per run. A step is ONE C-ABI call,
ospf_sweep_run (include/openr_spf.h): the library owns the path, the width
classes, their streams and the HIP graph it replays. Ranks (one process per
GPU) run the parts of the library's root partition, so the total work per
step is fixed: scaling "strong"; for N > 1 the digest records are
all-gathered over RCCL each step. The digests are poisoned before the timed
loop and the last timed step's digests are checked against the CPU
restatements on a role-stratified root set (`parity_vs_cpu_sample`).

Other topologies (parity / side benches, not the headline): fabric10k,
fabric100k-w and fabric10k-w (metrics 1..64, seed 7: the weighted cover
path), grid31, grid100 (unit 100x100 grid, diameter 198), mesh1m (8,192
sampled roots on the per-class batch driver).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--topology T]
       torchrun --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \\
                --master-port P bench.py --gpus N ...
Profiling mode (one class alone, R launches on one stream, no JSON line):
       python bench.py --mode classes --class-only W --reps R
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
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
    if name == "grid100":
        return T.grid(100), "G100 grid 100x100 (unit metric, diameter 198)", False, 0
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


class BusySampler:
    """GPU activity during the timed region, independent of our own clocks:
    the amdgpu driver's gpu_busy_percent of this device (sysfs, by its PCI
    address) sampled every 5 ms on a host thread."""

    def __init__(self, dev_index: int):
        self.path = None
        self.vals = []
        try:
            p = torch.cuda.get_device_properties(dev_index)
            addr = f"{getattr(p, 'pci_domain_id', 0):04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
            cand = f"/sys/bus/pci/devices/{addr}/gpu_busy_percent"
            if os.path.exists(cand):
                self.path = cand
        except Exception:  # noqa: BLE001 -- evidence only; absent on some hosts
            self.path = None
        self._stop = threading.Event()
        self._t = None

    def _run(self):
        while not self._stop.is_set():
            try:
                with open(self.path) as f:
                    self.vals.append(int(f.read().strip()))
            except (OSError, ValueError):
                return
            self._stop.wait(0.005)

    def __enter__(self):
        if self.path:
            self._t = threading.Thread(target=self._run, daemon=True)
            self._t.start()
        return self

    def __exit__(self, *exc):
        self._stop.set()
        if self._t:
            self._t.join()
        BUSY["timed"] = self.summary()

    def summary(self):
        if not self.vals:
            return {"source": self.path, "samples": 0,
                    "note": "no gpu_busy_percent file for this device"}
        v = np.asarray(self.vals, dtype=np.float64)
        return {"source": self.path, "samples": int(v.size), "mean_pct": round(float(v.mean()), 1),
                "min_pct": int(v.min()), "max_pct": int(v.max()),
                "note": "amdgpu gpu_busy_percent of this device sampled every 5 ms over the timed "
                        "loop (the driver's counter, not our HIP events)"}


BUSY = {}


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
    ap.add_argument("--part-of", type=int, default=-1,
                    help="sweep one part of the all-sources sweep's root partition into K parts "
                         "(a contiguous block of the partition's order; the middle part), "
                         "K x N parts over N ranks; -1: mesh1m 122 (~8.2k roots), else off")
    ap.add_argument("--root-sample", choices=["random", "block"], default="random",
                    help="sampled roots (--roots / mesh1m): a random sample, or one block of "
                         "consecutive node ids (a contiguous slice of the all-sources sweep; "
                         "mesh ids follow a Hilbert curve)")
    ap.add_argument("--root-order", choices=["auto", "locality", "random"], default="auto",
                    help="sweep order within a width class: grouped by smallest neighbour "
                         "(multi-source batches share frontiers), the random permutation, or "
                         "auto = grouped for single-word classes only")
    ap.add_argument("--profile-dir", default=os.path.join(ROOT, "profiles", "r06"))
    ap.add_argument("--iso-reps", type=int, default=3,
                    help="isolated launches per class for the roofline (after the timed steps)")
    ap.add_argument("--class-only", type=int, default=0,
                    help="profiling mode: launch only the class with this neighbour capacity "
                         "(8, 16, or 32 x next-hop words)")
    ap.add_argument("--reps", type=int, default=3, help="launches in --class-only mode")
    ap.add_argument("--mode", choices=["auto", "derive", "wcover", "wderive", "wmulti", "batch", "lds",
                                       "classes"],
                    default="auto",
                    help="all-sources sweep path (ospf_sweep_opts.mode; auto = the engine's "
                         "choice); classes = the per-class batch driver below (no sweep)")
    ap.add_argument("--graph", choices=["auto", "on", "off"], default="auto",
                    help="sweeps: the library captures one run in a HIP graph and replays it "
                         "(auto: on; eager launches if capture fails)")
    ap.add_argument("--dist-parity", type=int, default=0,
                    help="N>1: rank 0 checks the gathered digests of the last timed step "
                         "for this many roots against the CPU restatement")
    ap.add_argument("--no-probe", action="store_true",
                    help="sweeps: skip the store-bandwidth probe beside the roofline")
    ap.add_argument("--ab", default="",
                    help='sweeps: in-process A/B of engine env knobs, e.g. "OSPF_LEAF_CTILES=20;'
                         'OSPF_LEAF_GROUP_MAJOR=1" (variants ";"-separated, settings ",")')
    ap.add_argument("--ab-rounds", type=int, default=3)
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
    if args.part_of < 0:
        args.part_of = 122 if (args.topology == "mesh1m" and args.roots < 0) else 0
    if args.part_of > 0:
        n_roots = 0  # the part's roots, through the sweep
    sweep_ok = (n_roots <= 0 and args.roots_per_gpu == 0 and not args.no_nh
                and not args.class_only and args.mode != "classes")
    if sweep_ok:
        return sweep_main(args, eng, csr, names, stream, desc, V, E, world, rank, dist_on, dev,
                          backend, coll_dev)
    pool = perm if n_roots <= 0 else perm[: min(n_roots, V)]
    if n_roots > 0 and args.root_sample == "block":  # ids [V/2 - n/2, V/2 + n/2)
        k = min(n_roots, V)
        pool = np.arange(V // 2 - k // 2, V // 2 - k // 2 + k, dtype=np.uint32)
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
            m = c.roots.size  # (a class smaller than the world: one root per rank < m)
            x["slot"] = min(c.per_step, max(1, m // world))
            x["n"] = x["slot"] if m >= world else (1 if rank < m else 0)
        else:  # strong: this rank's contiguous slice of the class, every step
            lo, hi = shard.rank_slice(c.roots.size, world, rank)
            x["mine"] = c.roots[lo:hi]
            x["n"] = hi - lo
            x["slot"] = -(-c.roots.size // world)  # gather slot per rank (padded)
    classes = [c for c in classes if c.extra["slot" if weak else "n"] > 0]
    B = sum(c.extra["n"] for c in classes)
    B_all = B
    if dist_on and weak:  # ranks may run different counts (classes smaller than the world)
        t = torch.tensor([B], dtype=torch.int64, device=coll_dev)
        torch.distributed.all_reduce(t)
        B_all = int(t.item())
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
                    start = rank if c.roots.size < world else \
                        ((i * world + rank) * n) % c.roots.size
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
    with BusySampler(torch.cuda.current_device()):
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

    roots_total = B_all * args.steps if weak else pool.size * args.steps

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
    report(args, stream, names, csr, step_digest, dt, roots_total, E, desc, n_roots, V, world,
           rank, dist_on, backend, int(B_all if weak else pool.size), classes_cfg, roofline,
           "weak" if weak else "strong", "batch", pool=pool)
    if dist_on:
        torch.distributed.destroy_process_group()


def sweep_main(args, eng, csr, names, stream, desc, V, E, world, rank, dist_on, dev, backend,
               coll_dev):
    """All-sources step through the library's sweep (ospf_sweep_*, include/
    openr_spf.h): one C-ABI call per step, ospf_sweep_run, queues the whole
    sweep -- the path the engine picks for the graph (derive: distance-only
    128-root BFS + next hops from neighbours' level rows; wcover: cover SPF +
    leaf / cover next-hop derivation; wderive / batch), its width classes on
    their streams, replayed from one HIP graph. Rank r runs part r of the
    library's root partition (pod / plane blocks on a fabric); for N > 1 the
    24-B digests are all-gathered over RCCL each step."""
    mode = {"auto": "auto", "derive": "derive", "batch": "batch"}.get(args.mode, args.mode)
    K = max(1, args.part_of)
    part, n_parts = (K // 2) * world + rank, world * K  # K = 1: rank of world
    t0 = time.time()
    sw = eng.sweep(mode=mode, part=part, n_parts=n_parts, hip_graph=args.graph != "off")
    create_s = time.time() - t0
    n = sw.n_roots
    log(f"[rank {rank}] sweep: mode {sw.mode}, {n} roots, {sw.n_rows} rows, {sw.n_launches} "
        f"launches, hip graph {'on' if sw.hip_graph else 'off'}, "
        f"{sw.device_bytes / 2**30:.1f} GiB in {time.time() - t0:.1f}s")
    main_s = torch.cuda.current_stream()
    slot = n
    if dist_on:  # padded gather slots; every rank's root order, once
        t = torch.tensor([n], dtype=torch.int64, device=coll_dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        slot = int(t.item())
        rbuf = torch.full((slot,), -1, dtype=torch.int64, device=dev)
        rbuf[:n] = torch.from_numpy(sw.roots.astype(np.int64)).to(dev)
        groots = shard.gather_digests(rbuf.view(-1, 1).repeat(1, 3))[:, 0].cpu().numpy()
        groots = groots.reshape(world, slot)
    gbuf = torch.zeros((max(1, slot), 3), dtype=torch.int64, device=dev)
    gathered = {}

    def step():
        sw.run(main_s.cuda_stream)
        if dist_on:
            sw.digests_dev(gbuf.data_ptr(), main_s.cuda_stream)
            gathered["g"] = shard.gather_digests(gbuf)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    eng.sync(main_s.cuda_stream)
    # every digest the runs write set to 0xFF: a timed run that computed
    # nothing (an empty graph replay) fails the parity check below
    sw.poison(main_s.cuda_stream)
    gbuf.fill_(-1)
    torch.cuda.synchronize()
    if dist_on:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    with BusySampler(torch.cuda.current_device()):
        t_start = time.perf_counter()
        for _ in range(args.steps):
            step()
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
    if dist_on:
        g = gathered["g"].cpu().numpy().view(np.uint64).reshape(world, slot, 3)
        for r in range(world):
            for j, root in enumerate(groots[r]):
                if root >= 0:
                    step_digest[int(root)] = g[r, j]
    else:
        sw.digests_dev(gbuf.data_ptr(), main_s.cuda_stream)
        d = gbuf.cpu().numpy().view(np.uint64)
        for j, root in enumerate(sw.roots):
            step_digest[int(root)] = d[j]

    # every launch alone on its stream (HIP events there, inside the library)
    prof = sw.profile(args.iso_reps)
    units = []
    for p in prof:
        sec = p["ms_median"] / 1e3
        tr = pmc_traffic(args.profile_dir, p["name"], p["n_roots"])
        units.append({"launch": p["name"], "kernel": p["kernel"], "roots_per_launch": p["n_roots"],
                      "nh_words": p["nh_words"], "isolated_launch_ms": round(p["ms_median"], 3),
                      "isolated_launch_ms_min": round(p["ms_min"], 3),
                      "compulsory_bytes": p["compulsory_bytes"],
                      "achieved": round(p["compulsory_bytes"] / sec / 1e9, 1),
                      "frac": round(p["compulsory_bytes"] / sec / 1e9 / HBM_PEAK_GBS, 4),
                      "traffic": tr,
                      "traffic_over_compulsory": round(tr / p["compulsory_bytes"], 2)
                      if tr else None})
    dom = max(units, key=lambda u: u["isolated_launch_ms"])
    step_s = dt / args.steps
    roofline = {
        "bound": "hbm", "achieved": dom["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": dom["frac"], "traffic": dom["traffic"], "kernel": dom["kernel"],
        "launch": dom["launch"], "roots_per_launch": dom["roots_per_launch"],
        "avg_launch_ms": dom["isolated_launch_ms"], "compulsory_bytes": dom["compulsory_bytes"],
        "traffic_over_compulsory": dom["traffic_over_compulsory"], "launches": units,
        "step_compulsory_bytes": sw.step_compulsory_bytes,
        "step_frac": round(sw.step_compulsory_bytes / step_s / 1e9 / HBM_PEAK_GBS, 4),
        "note": "achieved = compulsory bytes of the dominant launch / its isolated time (median "
                "of HIP-event-timed launches alone on its stream, ospf_sweep_profile): levels = "
                "dist rows written (4V per run) + one neighbour-id + offset scan per 128-root "
                "traversal; derive = next-hop rows written (4VW per run); cover_spf = dist rows "
                "+ one weighted CSR scan; wderive = leaf dist + next-hop rows + cover rows read "
                "once. Level rows are intermediate (traffic, not compulsory). step_frac = the "
                "sweep's compulsory bytes / ms_per_step. traffic = measured HBM bytes per launch "
                "(rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, profiles/<round>/pmc_traffic.json)",
    }
    cfg = {"mode": sw.mode, "hip_graph": sw.hip_graph, "roots_this_rank": n,
           "rows_this_rank": sw.n_rows, "device_bytes": sw.device_bytes,
           "closure_over_roots": round(sw.n_rows / max(1, n), 4),
           "sweep_create_ms": round(create_s * 1e3, 1),
           "sweep_create_note": "ospf_sweep_create: host plan (partition, leaf set, twin "
                                "classes, row positions), allocation, one eager run and the HIP "
                                "graph capture; paid once per graph version, not in `value`"}
    trav = sw.step_traversed_edges
    sw_roots = sw.roots.copy()
    sw.close()
    # what a production caller pays once per graph version (odl::LinkState:
    # a deferred create -- plan + allocation -- then one eager run)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    sw2 = eng.sweep(mode=mode, part=part, n_parts=n_parts, defer=True)
    t2 = time.perf_counter()
    sw2.run(main_s.cuda_stream)
    torch.cuda.synchronize()
    eng.sync(main_s.cuda_stream)
    t3 = time.perf_counter()
    sw2.close()
    cfg["first_sweep_after_graph_change"] = {
        "plan_ms": round((t2 - t1) * 1e3, 1), "first_run_ms": round((t3 - t2) * 1e3, 1),
        "total_ms": round((t3 - t1) * 1e3, 1),
        "note": "a new graph version: ospf_sweep_create(OSPF_SWEEP_DEFER) + the first (eager, "
                "no HIP graph) run, as odl::LinkState::prefetchAllSources pays it"}
    # the store probe after the first-sweep record: its 67 GB buffer freed just
    # before that record had stalled the deferred sweep's first allocation by
    # ~3.7 s on some boxes (profiles/r06/f4_first_run_check)
    probe = store_probe(eng, V, dom, args) if not args.no_probe else None
    if probe:
        roofline["store_probe"] = probe
        best = max(probe.get("stream_GBs") or 0.0, probe.get("rows_chunk_GBs") or 0.0,
                   probe.get("rows_group_GBs") or 0.0)
        if best > 0:
            roofline["frac_of_box_store_rate"] = round(dom["achieved"] / best, 4)
    if args.ab:
        roofline["ab"] = ab_sweeps(args, eng, mode, part, n_parts, main_s, step_digest, sw_roots)
    if K > 1:  # one part per rank of a K x N partition: the parts' roots, not V
        tot = n
        if dist_on:
            t = torch.tensor([n], dtype=torch.int64, device=coll_dev)
            torch.distributed.all_reduce(t)
            tot = int(t.item())
        cfg["part_of"] = {"parts": n_parts, "part_of_rank0": (K // 2) * world,
                          "roots_all_ranks": tot,
                          "note": "a contiguous block of the all-sources sweep's root partition "
                                  "(each width class in largest-neighbour order, cut into "
                                  "n_parts slices); value = its roots / step time"}
        report(args, stream, names, csr, step_digest, dt, tot * args.steps, E, desc, tot, V,
               world, rank, dist_on, backend, tot, cfg, roofline, "strong", "sweep:" + cfg["mode"],
               pool=np.sort(sw_roots), trav_edges=trav * args.steps,
               scope=f" part {(K // 2) * world} .. +{world} of {n_parts} of the all-sources sweep "
                     f"({tot} roots)")
    else:
        report(args, stream, names, csr, step_digest, dt, V * args.steps, E, desc, 0, V, world,
               rank, dist_on, backend, V, cfg, roofline, "strong", "sweep:" + cfg["mode"],
               trav_edges=trav * args.steps)
    if dist_on:
        torch.distributed.destroy_process_group()


def store_probe(eng, V: int, dom: dict, args):
    """The box's own HBM store rate beside the dominant launch
    (ospf_probe_store, HIP events): the same bytes as the dominant launch's
    dist + next-hop rows -- `rows` = its roots -- written (0) in address
    order, (1) in the leaf launch's block shape, chunk-major, (2) the same
    group-major. A slow box shows in all three; a code regression only in
    the launch's own time."""
    if V % 4 or dom["roots_per_launch"] <= 0:
        return None
    rows = int(dom["roots_per_launch"])
    P = (V + 31) // 32 * 32 if os.environ.get("OSPF_SWEEP_ROW_PITCH", "") != "V" else V
    out = {"bytes": 2 * rows * P * 4, "rows": rows, "row_pitch_words": P, "group": 48,
           "ctiles": 6,
           "note": "ospf_probe_store: 16-B non-temporal stores of 2 x rows x pitch u32 (the dominant "
                   "launch's dist + next-hop rows at the sweep's row pitch: V rounded up to 32 "
                   "words, 128-B aligned rows), median of 3 HIP-event-timed launches after one "
                   "untimed; rows_* = blocks of 48 rows x 6 tiles of 1,024 nodes, the leaf "
                   "launch's shape"}
    for pat in ("stream", "rows_chunk", "rows_group"):
        try:
            ms = float(np.median(eng.probe_store(pat, P, rows, 48, 6, reps=3)))
        except Exception as e:  # noqa: BLE001 -- evidence only (e.g. no room beside the sweep)
            out[pat + "_error"] = str(e)
            continue
        out[pat + "_ms"] = round(ms, 3)
        out[pat + "_GBs"] = round(out["bytes"] / (ms / 1e3) / 1e9, 1)
    return out


def ab_sweeps(args, eng, mode, part, n_parts, main_s, base_digest, roots):
    """In-process A/B of engine knobs (env variables read when a sweep is
    created / captured): `--ab "A=1;B=2,C=3"` times the base sweep and each
    variant, interleaved over --ab-rounds rounds, each `--steps` replays,
    and checks every variant's digests against the base run's timed step."""
    variants = [""] + [v for v in args.ab.split(";") if v.strip()]
    res = {v or "base": [] for v in variants}
    parity = {}
    for _ in range(args.ab_rounds):
        for v in variants:
            saved = {}
            for kv in filter(None, v.split(",")):
                k, val = kv.split("=", 1)
                saved[k] = os.environ.get(k)
                os.environ[k] = val
            try:
                sw = eng.sweep(mode=mode, part=part, n_parts=n_parts, hip_graph=args.graph != "off")
                for _w in range(2):
                    sw.run(main_s.cuda_stream)
                torch.cuda.synchronize()
                sw.poison(main_s.cuda_stream)
                torch.cuda.synchronize()
                t = time.perf_counter()
                for _s in range(args.steps):
                    sw.run(main_s.cuda_stream)
                torch.cuda.synchronize()
                res[v or "base"].append((time.perf_counter() - t) / args.steps * 1e3)
                eng.sync(main_s.cuda_stream)
                g = torch.zeros((max(1, sw.n_roots), 3), dtype=torch.int64, device=main_s.device)
                sw.digests_dev(g.data_ptr(), main_s.cuda_stream)
                d = g.cpu().numpy().view(np.uint64)
                ok = all(np.array_equal(d[j], base_digest[int(r)]) for j, r in enumerate(sw.roots)
                         if int(r) in base_digest)
                parity[v or "base"] = parity.get(v or "base", True) and bool(ok)
                sw.close()
            finally:
                for k, old in saved.items():
                    if old is None:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = old
    return [{"env": k, "ms_per_step": [round(x, 3) for x in ms],
             "ms_median": round(float(np.median(ms)), 3), "digests_equal_base": parity.get(k)}
            for k, ms in res.items()]


def parity_sample(csr, V: int, k: int = 256):
    """Role-stratified parity roots: every width class (by distinct neighbours:
    8 / 16 / 32 x next-hop words; on a fabric racks, fabric switches and
    spines) whole when it has <= 2k members, else k drawn with seed 0x5eed."""
    nb = shard.distinct_neighbors(csr["row_ptr"], csr["col"])
    caps = shard.neighbor_caps(nb)
    rng = np.random.default_rng(SEED)
    out = []
    for cap in sorted(set(caps.tolist())):
        m = np.nonzero(caps == cap)[0].astype(np.uint32)
        out.append(m if m.size <= 2 * k else np.sort(rng.choice(m, k, replace=False)))
    return np.concatenate(out) if out else np.zeros(0, np.uint32)


def report(args, stream, names, csr, step_digest, dt, roots_total, E, desc, n_roots, V, world,
           rank, dist_on, backend, roots_per_step, classes_cfg, roofline, scaling, mode,
           pool=None, trav_edges=None, scope=None):
    """CPU baseline + parity of the timed step's digests (rank 0) and the one
    JSON line. gteps = edges the traversal kernels relaxed (trav_edges over
    the timed steps; every root of a per-root / batch path traverses E) / t;
    gteps_all_pairs_equiv = roots x E_dir / t, what per-root SSSPs would have
    to relax for the same rows (derived rows relax none)."""
    spf_s = roots_total / dt
    gteps_eq = roots_total * E / dt / 1e9
    gteps = (trav_edges if trav_edges is not None else roots_total * E) / dt / 1e9
    cpu = parity = None
    perm = np.random.default_rng(SEED).permutation(V).astype(np.uint32)
    if pool is None:
        pool = perm
    strat = parity_sample(csr, V) if n_roots <= 0 else pool[:256]
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
        # CSR-Dijkstra restatement: the role-stratified parity roots (every
        # spine of a fabric, 256 fabric switches, 256 racks) + the baseline's
        csr_ids = sorted(set(int(r) for r in strat) | set(sample_ids)) if not mesh else \
            [int(r) for r in pool[:64]]
        t1 = time.perf_counter()
        fd = o.fast_digests([names[i] for i in csr_ids], threads=threads)
        ct_fast = time.perf_counter() - t1
        csr_line = {"value": round(len(csr_ids) / ct_fast, 3), "unit": "SPF/s",
                    "cores": threads, "kind": "port",
                    "sample": f"{len(csr_ids)} roots (role-stratified parity set + the "
                              f"baseline's), CSR-Dijkstra restatement (oracle/, integer ids, "
                              f"binary heap), {threads} threads, {ct_fast:.2f}s"}
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
            nb = shard.distinct_neighbors(csr["row_ptr"], csr["col"])
            caps = shard.neighbor_caps(nb)
            by_cap = {}
            for r in checks:
                by_cap[int(caps[r])] = by_cap.get(int(caps[r]), 0) + 1
            parity = {"roots": len(checks),
                      "roots_by_neighbour_class": {str(c_): v for c_, v in sorted(by_cap.items())},
                      "equal": bool(all(r in step_digest and np.array_equal(step_digest[r], d)
                                        for r, d in checks.items())),
                      "source": "digests of the last timed step (poisoned with 0xFF before the "
                                "timed loop) vs the CPU restatement(s)"}

    if rank == 0 and dist_on and args.dist_parity > 0 and step_digest:
        from oracle import Oracle  # checker only, after the timed region
        k = min(args.dist_parity, len(strat))  # spread over the width classes
        ids = [int(r) for r in strat[np.linspace(0, len(strat) - 1, k).astype(np.int64)]]
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
            "gteps_all_pairs_equiv": round(gteps_eq, 3),
            "gteps_note": "gteps = edges relaxed by the traversal kernels per second (seed BFS "
                          "rows x E_dir, or the cover Dial's rows x contracted edges; rows "
                          "derived from neighbours' rows relax no edge); gteps_all_pairs_equiv "
                          "= roots x E_dir / t (not work done)",
            "config": {
                "workload": desc + (scope if scope else " all-sources" if n_roots <= 0 else
                                    f" {pool.size} sampled roots") +
                " SPF + ECMP next-hop bitsets (dist + next-hop rows written to HBM, per-root "
                "digests)",
                "n_nodes": V, "n_directed_edges": E, "mode": mode,
                "roots_per_step": roots_per_step,
                "root_sample": "partition part" if scope else
                               args.root_sample if n_roots > 0 else "all",
                "root_classes": classes_cfg,
                "parallelism": f"root-sharded x{world}" +
                               (f", all_gather of 24-B digests ({'RCCL' if backend == 'nccl' else backend})"
                                if dist_on else "")},
            "roofline": roofline, "cpu_baseline": cpu, "parity_vs_cpu_sample": parity,
            "gpu_busy": BUSY.get("timed"),
        }
        if dist_on:
            line["gathered_roots"] = len(step_digest)
            line["dist_backend"] = backend
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
