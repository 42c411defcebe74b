"""openr_amd — MI355X-native batched SPF engine for OpenR's Decision module.

Scope: the LinkState SPF hot path only —
``LinkState::runSpf / getSpfResult / getKthPaths`` (openr/decision/LinkState.cpp)
re-built as hand-written CDNA4 HIP kernels behind a C ABI
(include/openr_spf.h), with a host-side C++ LinkState mirror
(include/openr_decision.h) that keeps the reference's API and semantics.

Modules:
  adjdb      AdjacencyDatabase update streams (input format)
  topology   grid / fabric / mesh generators (RoutingBenchmarkUtils shapes)
  engine     ``Engine``: the C-ABI SPF engine (CSR in HBM, batched roots)
  linkstate  ``LinkState``: GPU-backed LinkState mirror
  build      in-tree native build (hipcc, gfx950)
"""
from .adjdb import AdjDb, AdjDbStream, Adjacency, create_adjacency  # noqa: F401

__all__ = ["AdjDb", "AdjDbStream", "Adjacency", "create_adjacency"]
