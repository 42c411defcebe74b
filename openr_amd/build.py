"""Build the native libraries in-tree (gfx950 only).

  openr_amd/lib/libopenr_spf_hip.so  — HIP engine (include/openr_spf.h)
  openr_amd/lib/libopenr_decision.so — host LinkState mirror (include/openr_decision.h)

Run: python -m openr_amd.build   (or __graft_entry__.build()).
"""
from __future__ import annotations

import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
LIB = os.path.join(PKG, "lib")
ENGINE_SRC = [os.path.join(PKG, "csrc", "engine", f) for f in ("spf_kernels.hip", "spf_bfs.hip", "spf_msbfs.hip", "spf_ksp2.hip", "spf_dial.hip", "spf_wdial.hip", "spf_wderive.hip", "spf_levels.hip", "spf_cover.hip", "spf_update.hip",
                                                                 "spf_engine.hip")]
DECISION_SRC = [os.path.join(PKG, "csrc", "decision", f)
                for f in ("link_state.cpp", "spf_solver.cpp", "decision_capi.cpp")]
ENGINE_SO = os.path.join(LIB, "libopenr_spf_hip.so")
DECISION_SO = os.path.join(LIB, "libopenr_decision.so")
HEADERS = [os.path.join(ROOT, "include", h)
           for h in ("openr_spf.h", "openr_decision.h", "openr_adjdb.h")] + \
    [os.path.join(PKG, "csrc", "engine", "spf_kernels.h"),
     os.path.join(PKG, "csrc", "decision", "link_state.h"),
     os.path.join(PKG, "csrc", "decision", "spf_solver.h")]

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"


def _stale(out, srcs):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(s) > t for s in srcs + HEADERS)


def _run(cmd):
    print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)


def build(force: bool = False, verbose_resources: bool = False) -> None:
    os.makedirs(LIB, exist_ok=True)
    if force or _stale(ENGINE_SO, ENGINE_SRC):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
               "-Wall", "-Wno-unused-result", "-o", ENGINE_SO] + ENGINE_SRC
        if verbose_resources:
            cmd.insert(1, "-Rpass-analysis=kernel-resource-usage")
        _run(cmd)
    if force or _stale(DECISION_SO, DECISION_SRC + [ENGINE_SO]):
        _run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-Wextra",
              "-Wno-unused-parameter", "-o", DECISION_SO] + DECISION_SRC +
             ["-L" + LIB, "-lopenr_spf_hip", "-Wl,-rpath,$ORIGIN"])


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose_resources="--resources" in sys.argv)
