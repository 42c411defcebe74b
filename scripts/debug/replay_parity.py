#!/usr/bin/env python3
"""Debug: digests of a sweep after poison + N graph replays vs the first run and
vs the CSR-Dijkstra restatement, per width class, for a few env variants.
Usage: python scripts/debug/replay_parity.py [--topology fabric10k-w|mesh] [--mode auto]"""
import argparse
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def one(topo, mode, hip_graph, reps, part_of):
    import numpy as np
    import torch  # noqa: F401
    from oracle import Oracle
    from openr_amd import topology as T
    from openr_amd.engine import Engine, Sweep
    from openr_amd.linkstate import LinkState
    if topo == "fabric10k-w":
        st = T.fabric(pods=173, planes=8, weighted_seed=7)
    elif topo == "fabric100k-w":
        st = T.fabric(pods=1781, planes=8, weighted_seed=7)
    else:
        st = T.mesh(int(topo.split(":")[1]) if ":" in topo else 100000, seed=42)
    ls = LinkState()
    ls.apply(st)
    names = ls.node_names()
    csr = ls.csr()
    eng = Engine()
    eng.load(csr)
    V = eng.V
    part, n_parts = (part_of // 2, part_of) if part_of > 1 else (0, 1)
    sw = Sweep(eng, mode=mode, hip_graph=hip_graph, part=part, n_parts=n_parts)

    def digs():
        d = np.zeros((max(1, sw.n_roots), 3), np.uint64)
        sw._check(sw._L.ospf_sweep_digests_host(sw._h, d.ctypes.data))
        return d[: sw.n_roots].copy()
    first = digs()
    if hip_graph:
        nm, nd, no = sw.graph_memsets()
        print(f"captured memset nodes {nm}: dst outside every live allocation {nd}, "
              f"inside the sweep's own blocks {no}", flush=True)
    s = torch.cuda.current_stream()
    if not os.environ.get("RP_NOPOISON"):
        sw.poison(s.cuda_stream)
    for _ in range(reps):
        sw.run(s.cuda_stream)
    eng.sync(s.cuda_stream)
    last = digs()
    roots = sw.roots
    rng = np.random.default_rng(1)
    pick = np.sort(rng.choice(np.arange(roots.size), min(400, roots.size), replace=False))
    want = Oracle(st).fast_digests([names[roots[j]] for j in pick], True, threads=16)
    nb = np.array([eng.nh_words(int(r)) for r in roots])
    bad_first = np.nonzero(~np.all(first[pick] == want, axis=1))[0]
    bad_last = np.nonzero(~np.all(last[pick] == want, axis=1))[0]
    drift = np.nonzero(~np.all(first == last, axis=1))[0]
    print(f"{topo} mode={sw.mode} graph={sw.hip_graph} env="
          f"{ {k: v for k, v in os.environ.items() if k.startswith('OSPF_')} } rows={sw.n_rows}: "
          f"first-run bad {len(bad_first)}/{len(pick)} (W {sorted(set(nb[pick[bad_first]].tolist()))}), "
          f"after {reps} replays bad {len(bad_last)} (W {sorted(set(nb[pick[bad_last]].tolist()))}), "
          f"first != last {len(drift)} (W {sorted(set(nb[drift].tolist()))})", flush=True)
    if len(drift):
        j = drift[0]
        print("   e.g. root", names[roots[j]], "first", first[j], "last", last[j], flush=True)
    sw.close()
    eng.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--topology", default="fabric10k-w")
    ap.add_argument("--mode", default="auto")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--part-of", type=int, default=0)
    ap.add_argument("--variants", default="base,graphoff,seednonh,closurenonh")
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--graph", type=int, default=1)
    a = ap.parse_args()
    if a.child:
        one(a.topology, a.mode, bool(a.graph), a.reps, a.part_of)
        return
    envs = {"base": ({}, 1), "graphoff": ({}, 0), "seednonh": ({"OSPF_SEED_NONH": "1"}, 1),
            "closurenonh": ({"OSPF_CLOSURE_NONH": "1"}, 1),
            "zerok": ({"OSPF_ZERO_KERNEL": "1"}, 1),
            "memset": ({"OSPF_ZERO_MEMSET": "1"}, 1), "memsetoff": ({"OSPF_ZERO_MEMSET": "1"}, 0), "nopoison": ({"RP_NOPOISON": "1"}, 1)}
    for v in a.variants.split(","):
        e, g = envs[v]
        env = dict(os.environ, **e)
        r = subprocess.run([sys.executable, "-u", __file__, "--child", "--topology", a.topology,
                            "--mode", a.mode, "--reps", str(a.reps), "--graph", str(g),
                            "--part-of", str(a.part_of)], env=env, timeout=600)
        if r.returncode:
            print(f"variant {v} rc={r.returncode}", flush=True)
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
