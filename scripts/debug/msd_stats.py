#!/usr/bin/env python3
"""Debug: the WMULTI sweep of a mesh part, timed per unit, with the msdist
phase / visit counters (OSPF_MSD_STATS) for a few bucket widths.
Usage: python scripts/debug/msd_stats.py [--points 1000000] [--part-of 122] [--deltas 16,64,256]"""
import argparse
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def child(points, part_of, reps):
    import torch  # noqa: F401
    from openr_amd import topology as T
    from openr_amd.engine import Engine, Sweep
    from openr_amd.linkstate import LinkState
    st = T.mesh(points, seed=42)
    ls = LinkState()
    ls.apply(st)
    eng = Engine()
    eng.load(ls.csr())
    t0 = time.time()
    sw = Sweep(eng, mode="wmulti", hip_graph=False, defer=True, part=part_of // 2, n_parts=part_of)
    print(f"plan {time.time() - t0:.2f}s roots {sw.n_roots} rows {sw.n_rows}", flush=True)
    t0 = time.time()
    sw.run()
    eng.sync()
    print(f"first run {time.time() - t0:.2f}s", flush=True)
    for p in sw.profile(reps):
        print(f"  {p['name']:>16} {p['n_roots']:6d} {p['ms_median']:9.2f} ms", flush=True)
    sw.close()
    eng.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=1_000_000)
    ap.add_argument("--part-of", type=int, default=122)
    ap.add_argument("--deltas", default="16,64")
    ap.add_argument("--reps", type=int, default=1)
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if a.child:
        child(a.points, a.part_of, a.reps)
        return
    for dl in a.deltas.split(","):
        env = dict(os.environ, OSPF_MSD_STATS="1", OSPF_MSD_DELTA=dl)
        print(f"--- delta {dl}", flush=True)
        r = subprocess.run([sys.executable, "-u", __file__, "--child", "--points", str(a.points),
                            "--part-of", str(a.part_of), "--reps", str(a.reps)], env=env,
                           timeout=900)
        if r.returncode:
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
