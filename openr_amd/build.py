"""Build the native libraries in-tree (gfx950 only).

  openr_amd/lib/libopenr_spf_hip.so  — HIP engine (include/openr_spf.h)
  openr_amd/lib/libopenr_decision.so — host LinkState mirror (include/openr_decision.h)

Each engine source is compiled to its own object (openr_amd/lib/obj/, in
parallel, only when it or a header changed), then linked.

Run: python -m openr_amd.build   (or __graft_entry__.build()).
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
LIB = os.path.join(PKG, "lib")
OBJ = os.path.join(LIB, "obj")
ENGINE_SRC = [os.path.join(PKG, "csrc", "engine", f)
              for f in ("spf_kernels.hip", "spf_bfs.hip", "spf_msbfs.hip", "spf_ksp2.hip",
                        "spf_dial.hip", "spf_wdial.hip", "spf_wderive.hip", "spf_levels.hip",
                        "spf_cover.hip", "spf_msdist.hip", "spf_update.hip", "spf_leaf.hip", "spf_twin.hip", "spf_small.hip",
                        "spf_probe.hip", "spf_engine.hip",
                        "spf_sweep.hip")]
DECISION_SRC = [os.path.join(PKG, "csrc", "decision", f)
                for f in ("link_state.cpp", "spf_solver.cpp", "adjdb_thrift.cpp", "decision_capi.cpp")]
ENGINE_SO = os.path.join(LIB, "libopenr_spf_hip.so")
DECISION_SO = os.path.join(LIB, "libopenr_decision.so")
HEADERS = [os.path.join(ROOT, "include", h)
           for h in ("openr_spf.h", "openr_decision.h", "openr_adjdb.h")] + \
    [os.path.join(PKG, "csrc", "engine", h) for h in ("spf_kernels.h", "spf_internal.h", "host_pool.h")]
DECISION_HEADERS = HEADERS + \
    [os.path.join(PKG, "csrc", "decision", h) for h in ("link_state.h", "spf_solver.h", "adjdb_thrift.h")]

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
JOBS = max(1, min(16, int(os.environ.get("MAX_JOBS", "0") or 0) or (os.cpu_count() or 4)))


def _newer(out, srcs):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.exists(s) and os.path.getmtime(s) > t for s in srcs)


def _run(cmd):
    print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)


def _obj(src):
    return os.path.join(OBJ, os.path.basename(src) + ".o")


def build(force: bool = False, verbose_resources: bool = False) -> None:
    os.makedirs(OBJ, exist_ok=True)
    todo = [s for s in ENGINE_SRC if force or _newer(_obj(s), [s] + HEADERS)]

    def compile_one(src):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
               "-Wno-unused-result", "-c", "-o", _obj(src)]
        if src.endswith(".cpp"):
            cmd += ["-x", "hip"]
        if verbose_resources:
            cmd.insert(1, "-Rpass-analysis=kernel-resource-usage")
        _run(cmd + [src])

    if todo:
        with ThreadPoolExecutor(JOBS) as ex:
            list(ex.map(compile_one, todo))
    objs = [_obj(s) for s in ENGINE_SRC]
    if force or todo or _newer(ENGINE_SO, objs):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", ENGINE_SO] + objs +
             ["-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"])
    if force or _newer(DECISION_SO, DECISION_SRC + DECISION_HEADERS + [ENGINE_SO]):
        _run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-Wextra",
              "-Wno-unused-parameter", "-o", DECISION_SO] + DECISION_SRC +
             ["-L" + LIB, "-lopenr_spf_hip", "-Wl,-rpath,$ORIGIN"])


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose_resources="--resources" in sys.argv)
