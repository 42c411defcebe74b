#!/usr/bin/env python3
"""Benchmark: all-sources SPF + ECMP next-hops on the 100k-node fabric.

BASELINE.json metric: "all-sources SPF/sec + GTEPS on 100k-node fabric
topology at 1/2/4/8 GPUs". A *step* = one batch of roots per GPU run through
the engine (ospf_sssp_batch_dev): per-root distances, next-hop bitsets and
digests written to HBM, then (N > 1) the 24-B per-root digest records
all-gathered over RCCL. Roots sweep a fixed permutation of every node (all
sources), grouped per launch by next-hop width class (RSW / FSW / SSW).
Roots are sharded across ranks with no data-path collective: scaling "weak".

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
       torchrun --nproc-per-node N bench.py --gpus N ...
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
    if name == "grid31":
        return T.grid(31), "G31 grid 31x31 (unit metric)"
    if name == "mesh1m":
        return T.mesh(1_000_000, seed=42), "M1M random-geometric mesh (metric 1..16)"
    raise SystemExit(f"unknown topology {name}")


def bytes_per_root(V: int, E: int, W: int) -> int:
    """CSR neighbour+weight reads, offsets, dist write,
    next-hop bitset write."""
    return 8 * E + 4 * (V + 1) + 4 * V + 4 * V * W


def pmc_traffic(profile_dir: str, kernel_substr: str):
    """Per-launch HBM bytes from committed rocprofv3 --pmc summaries
    (FETCH_SIZE x2 per the gfx950 correction + WRITE_SIZE, KiB units)."""
    path = os.path.join(profile_dir, "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get(kernel_substr)
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=1024, help="roots per GPU per step")
    ap.add_argument("--topology", default="fabric100k")
    ap.add_argument("--cpu-sample", type=int, default=32)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-nh", action="store_true", help="skip next-hop output (diagnostic)")
    ap.add_argument("--profile-dir", default=os.path.join(ROOT, "profiles", "r01"))
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist_on = world > 1
    if dist_on:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

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
        f"lds/block={getattr(props, 'shared_memory_per_block', '?')} "
        f"lds/cu={getattr(props, 'shared_memory_per_multiprocessor', '?')}")
    log(f"[rank {rank}] {desc}: V={V} E_dir={E} setup {time.time() - t0:.1f}s")

    # all-sources root permutation, grouped by next-hop width class
    rng = np.random.default_rng(0x5EED)
    perm = rng.permutation(V).astype(np.uint32)
    rp, col = csr["row_ptr"], csr["col"]
    deg_distinct = np.array([len(np.unique(col[rp[u]:rp[u + 1]])) for u in range(V)])
    words = np.maximum(1, (deg_distinct + 31) // 32)
    classes = []
    for W in sorted(set(words.tolist())):
        members = perm[words[perm] == W]
        share = max(1, int(round(args.batch * members.size / V)))
        classes.append(dict(W=W, roots=members, per_step=share))
    B = sum(c["per_step"] for c in classes)
    flags = N.OSPF_WANT_DIST | N.OSPF_WANT_DIGEST | (0 if args.no_nh else N.OSPF_WANT_NH)
    dev = torch.device("cuda", local)
    for c in classes:
        n = c["per_step"]
        c["d_all"] = torch.from_numpy(c["roots"].astype(np.int32)).to(dev)
        c["dist"] = torch.empty((n, V), dtype=torch.int32, device=dev)
        c["nh"] = None if args.no_nh else torch.empty((n, V, c["W"]), dtype=torch.int32, device=dev)
        c["dig"] = torch.empty((n, 3), dtype=torch.int64, device=dev)
        c["ms"] = []
        c["variant"] = eng.plan_variant(c["W"], flags)
    dig_all = torch.empty((B, 3), dtype=torch.int64, device=dev)
    gathered = torch.empty((world * B, 3), dtype=torch.int64, device=dev) if dist_on else None
    s = torch.cuda.current_stream()
    sh = s.cuda_stream
    # one HIP stream per root class so the classes' workgroups share the GPU
    # (the 3 spine roots are long single-root runs); heaviest class first
    for c in classes:
        c["stream"] = torch.cuda.Stream(device=dev)
        c["roots_i32"] = torch.empty(c["per_step"], dtype=torch.int32, device=dev)
    launch_order = sorted(classes, key=lambda c: -c["W"])

    def step(i: int, timed: bool):
        done_prev = torch.cuda.Event()
        done_prev.record(s)  # previous step's digest copies are queued on s
        for c in launch_order:
            n, m = c["per_step"], c["roots"].size
            start = ((i * world + rank) * n) % m
            cs = c["stream"]
            with torch.cuda.stream(cs):
                cs.wait_event(done_prev)
                idx = (torch.arange(n, device=dev) + start) % m
                torch.index_select(c["d_all"], 0, idx, out=c["roots_i32"])
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record(cs)
                eng.run_dev(c["roots_i32"].data_ptr(), n, c["W"], flags=flags,
                            d_dist=c["dist"].data_ptr(),
                            d_nh=c["nh"].data_ptr() if c["nh"] is not None else 0,
                            d_digest=c["dig"].data_ptr(), stream=cs.cuda_stream)
                ev[1].record(cs)
            if timed:
                c["ms"].append(ev)
        off = 0
        for c in classes:
            s.wait_event(c["ms"][-1][1] if timed else ev_record(c["stream"]))
            dig_all[off:off + c["per_step"]].copy_(c["dig"])
            off += c["per_step"]
        if dist_on:
            torch.distributed.all_gather_into_tensor(gathered, dig_all)

    def ev_record(cs):
        e = torch.cuda.Event()
        e.record(cs)
        return e

    for i in range(args.warmup):
        step(i, False)
    torch.cuda.synchronize()
    eng.sync(sh)
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
    eng.sync(sh)  # raises if the device error word was set
    if dist_on:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t.item())

    roots_total = world * B * args.steps
    spf_s = roots_total / dt
    gteps = roots_total * E / dt / 1e9

    # roofline for the dominant kernel (largest total device time)
    for c in classes:
        c["kernel_ms"] = [a.elapsed_time(b) for a, b in c["ms"]]
    dom = max(classes, key=lambda c: sum(c["kernel_ms"]))
    avg_ms = float(np.mean(dom["kernel_ms"]))
    alg_bytes = dom["per_step"] * bytes_per_root(V, E, dom["W"])
    achieved = alg_bytes / (avg_ms / 1e3) / 1e9
    kname = f"spf_run_kernel variant={dom['variant']} W={dom['W']}"
    roofline = {
        "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": pmc_traffic(args.profile_dir, f"W{dom['W']}"),
        "kernel": kname, "roots_per_launch": dom["per_step"],
        "bytes_per_root": bytes_per_root(V, E, dom["W"]),
        "avg_launch_ms": round(avg_ms, 3),
        "teps_per_launch": round(dom["per_step"] * E / (avg_ms / 1e3) / 1e9, 3),
    }

    cpu = None
    parity = None
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
        W = int(words[sample_ids].max())
        gd = eng.run(sample_ids, W, want_dist=False, want_nh=False, want_digest=True)["digest"]
        parity = bool(np.array_equal(gd, cd))

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(spf_s, 2), "unit": "SPF/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic", "gteps": round(gteps, 3),
            "config": {"workload": desc + " all-sources SPF + ECMP next-hop bitsets (dist+nh "
                                          "rows to HBM, per-root digests)",
                       "n_nodes": V, "n_directed_edges": E, "roots_per_step_per_gpu": B,
                       "root_classes": [{"nh_words": c["W"], "roots_per_step": c["per_step"],
                                         "variant": c["variant"]} for c in classes],
                       "parallelism": f"root-sharded x{world}" + (", RCCL all_gather of "
                                                                  "24-B digests" if dist_on else "")},
            "roofline": roofline, "cpu_baseline": cpu, "parity_vs_cpu_sample": parity,
        }
        print(json.dumps(line), flush=True)
    if dist_on:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
