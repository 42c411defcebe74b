"""Root sharding for multi-GPU all-sources runs.

Every SPF run is independent, so ranks split the roots with no data-path
collective; the only exchange is an all-gather of the fixed 24-byte per-root
digest records {reached, sum_dist, hash} (RCCL over xGMI on MI355X, gloo in
the CPU tests). Roots are grouped in next-hop width classes (one kernel launch
per class per step), and every class is swept round-robin over ranks.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Sequence

import numpy as np


@dataclass
class RootClass:
    nh_words: int
    roots: np.ndarray          # this class's roots in sweep order (u32 node ids)
    per_step: int              # roots of this class each rank runs per step
    extra: dict = field(default_factory=dict)
    cap: int = 0               # distinct-neighbour capacity of the class (8, 16, 32 W)


def neighbor_caps(nbrs: np.ndarray) -> np.ndarray:
    """Launch class of each root by its distinct-neighbour count: 8, 16, or
    32 x next-hop words. Classes of at most 8 / 16 neighbours let the engine
    use 8 / 16 bit-planes (multi-source BFS) or packed 32-bit state
    (weighted path) for the whole launch."""
    words = np.maximum(1, (nbrs + 31) // 32)
    return np.where(nbrs <= 8, 8, np.where(nbrs <= 16, 16, 32 * words)).astype(np.int64)


def nh_words_of(row_ptr: np.ndarray, col: np.ndarray) -> np.ndarray:
    """ceil(distinct neighbours / 32) per node (>= 1) from a CSR whose rows
    are sorted by neighbour id (what the engine uses for the bit order)."""
    return np.maximum(1, (distinct_neighbors(row_ptr, col) + 31) // 32)


def distinct_neighbors(row_ptr: np.ndarray, col: np.ndarray) -> np.ndarray:
    """Distinct neighbours per node (self-loops excluded) = next-hop bits a
    root needs (the engine's max_root_neighbors hint)."""
    V = row_ptr.size - 1
    deg = np.diff(row_ptr.astype(np.int64))
    owner = np.repeat(np.arange(V), deg)
    new = np.ones(col.size, bool)
    if col.size:
        new[1:] = (col[1:] != col[:-1]) | (owner[1:] != owner[:-1])
        new &= col != owner  # self-loops are not next hops
    return np.bincount(owner[new], minlength=V) if col.size else np.zeros(V, np.int64)


def first_neighbor(row_ptr: np.ndarray, col: np.ndarray) -> np.ndarray:
    """Smallest neighbour id per node (V for an isolated node)."""
    V = row_ptr.size - 1
    deg = np.diff(row_ptr.astype(np.int64))
    owner = np.repeat(np.arange(V), deg)
    key = np.full(V, V, np.int64)
    ok = col != owner
    np.minimum.at(key, owner[ok], col[ok].astype(np.int64))
    return key


def last_neighbor(row_ptr: np.ndarray, col: np.ndarray) -> np.ndarray:
    """Largest neighbour id per node (-1 for an isolated node): the derive
    mode's locality key (roots with the same largest neighbour tend to share
    most neighbours: a fabric's racks and fabric switches of one pod, the
    spines of one plane), so a block's group and its neighbours' level rows
    stay together in the caches."""
    V = row_ptr.size - 1
    deg = np.diff(row_ptr.astype(np.int64))
    owner = np.repeat(np.arange(V), deg)
    key = np.full(V, -1, np.int64)
    ok = col != owner
    np.maximum.at(key, owner[ok], col[ok].astype(np.int64))
    return key


def locality_order(roots: np.ndarray, key: np.ndarray) -> np.ndarray:
    """Roots grouped by their smallest neighbour (stable): roots hanging off
    the same hub share frontiers and next-hop planes in a multi-source batch,
    so one 64-root traversal does more useful work per edge it scans. Any
    order is valid for an all-sources sweep; this one is topology-agnostic."""
    return roots[np.argsort(key[roots], kind="stable")]


def make_classes(perm: np.ndarray, caps: np.ndarray, batch: int,
                 key: np.ndarray = None, max_grouped_words: int = None) -> List[RootClass]:
    """Split a root permutation into launch classes by `caps` (per node: the
    class's neighbour capacity, neighbor_caps, or 32 x next-hop words); each
    class's share of a `batch`-root step is
    proportional to its size (at least 1). With `key` (first_neighbor) the
    sweep of each class with at most `max_grouped_words` next-hop words (all
    classes when None) is locality-ordered."""
    V = perm.size
    out = []
    for cap in sorted(set(caps[perm].tolist())):
        members = perm[caps[perm] == cap]
        W = max(1, (int(cap) + 31) // 32)
        if key is not None and (max_grouped_words is None or W <= max_grouped_words):
            members = locality_order(members, key)
        share = max(1, int(round(batch * members.size / V)))
        out.append(RootClass(W, members.astype(np.uint32), share, cap=int(cap)))
    return out


def rank_slice(m: int, world: int, rank: int):
    """[lo, hi) of rank's contiguous share of m items (sizes differ by <= 1):
    the strong-scaling split of each width class over the ranks, so every
    root of an all-sources step runs exactly once."""
    q, r = divmod(m, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def step_roots(cls: RootClass, step: int, world: int, rank: int) -> np.ndarray:
    """Roots of `cls` that `rank` runs in `step` of a weak-scaling cyclic
    sweep; disjoint across ranks within a step (n <= m / world per rank; a
    class smaller than the world gives one root to each rank < m and none to
    the others)."""
    m = cls.roots.size
    if m < world:
        return cls.roots[[rank]] if rank < m else cls.roots[:0]
    n = min(cls.per_step, m // world)
    start = ((step * world + rank) * n) % m
    return cls.roots[(np.arange(n) + start) % m]


def gather_digests(local, group=None):
    """all_gather of per-rank [n, 3] int64 digest tensors -> [world*n, 3]."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    if dist.get_backend(group) == "nccl":  # RCCL on ROCm
        out = torch.empty((world * local.shape[0], 3), dtype=local.dtype, device=local.device)
        dist.all_gather_into_tensor(out, local, group=group)
        return out
    # gloo (CPU tests, or a multi-rank rehearsal sharing one GPU): host copies
    local = local.detach().cpu()
    parts = [torch.empty_like(local) for _ in range(world)]
    dist.all_gather(parts, local, group=group)
    return torch.cat(parts)


def ksp2_shards(V: int, neighbors: np.ndarray, world: int, rank: int):
    """scripts/bench_ksp2.py's split of one KSP2 + LFA step over ranks: a
    contiguous block of destination ids (np.array_split) and every world-th
    neighbour of the source for the LFA reruns. Disjoint and covering; the
    records need no collective (each rank holds its destinations' paths)."""
    dsts = np.array_split(np.arange(V, dtype=np.uint32), world)[rank]
    return dsts, np.asarray(neighbors)[rank::world]


def reassemble_by_destination(parts):
    """Merge per-rank {destination: record} maps (one per rank, disjoint) into
    one ordered by destination id."""
    out = {}
    for part in parts:
        for d, rec in part.items():
            if d in out:
                raise ValueError(f"destination {d} in two shards")
            out[d] = rec
    return dict(sorted(out.items()))


def digests_as_u64(t) -> np.ndarray:
    return t.cpu().numpy().view(np.uint64)


# ---------------------------------------------------------------- derive mode
# All-sources next hops from neighbour level rows (ospf_levels_dev +
# ospf_nh_derive_dev): a rank derives the next hops of its roots R from the
# level rows of R and of every neighbour of R, so it computes levels for the
# closure R + N(R). A partition whose slices are closed under most
# neighbourhoods keeps that duplication small.

def closure(roots: np.ndarray, row_ptr: np.ndarray, col: np.ndarray) -> np.ndarray:
    """Sorted node ids of roots and all their neighbours."""
    V = row_ptr.size - 1
    is_root = np.zeros(V, bool)
    is_root[roots] = True
    owner = np.repeat(np.arange(V), np.diff(row_ptr.astype(np.int64)))
    mark = is_root.copy()
    mark[col[is_root[owner]]] = True
    return np.nonzero(mark)[0].astype(np.uint32)


def fabric_partition(names: Sequence[str], world: int, rank: int):
    """Roots of `rank` for a fabric (topology.fabric names: SSW "1-plane-i",
    FSW "2-pod-plane", RSW "3-pod-i"): the racks and fabric switches of a
    contiguous block of pods and the spines of a contiguous block of planes.
    Its closure adds the 288 spines (next hops of its fabric switches) and
    the fabric switches of its planes in other pods (next hops of its
    spines): ~14% over 1/8 of the nodes at 8 ranks. None when the names are
    not a fabric's."""
    kind, a = [], []
    for nm in names:
        parts = nm.split("-")
        if len(parts) != 3 or parts[0] not in ("1", "2", "3"):
            return None
        t, x, y = int(parts[0]), int(parts[1]), int(parts[2])
        kind.append(t)
        a.append(x if t != 2 else x)  # pod (FSW, RSW) or plane (SSW)
    kind, a = np.array(kind), np.array(a)
    pods = int(a[kind != 1].max()) + 1 if np.any(kind != 1) else 1
    planes = int(a[kind == 1].max()) + 1 if np.any(kind == 1) else 1
    p0, p1 = rank_slice(pods, world, rank)
    q0, q1 = rank_slice(planes, world, rank)
    mine = ((kind != 1) & (a >= p0) & (a < p1)) | ((kind == 1) & (a >= q0) & (a < q1))
    return np.nonzero(mine)[0].astype(np.uint32)


# ---------------------------------------------------------------- weighted derive
# Weighted all-sources sweeps run a per-root SPF kernel for a vertex cover S
# of the graph and derive the rows of the other nodes -- an independent set I
# of "leaf" roots with <= 32 distinct neighbours, all in S -- from their
# neighbours' distance rows (ospf_wderive_dev). On the fabric I = the racks.

def leaf_set(row_ptr: np.ndarray, col: np.ndarray, max_nbrs: int = 32) -> np.ndarray:
    """Independent set of nodes with <= max_nbrs distinct neighbours, chosen
    greedily by (distinct neighbours, id): a node joins when it is the
    smallest undecided candidate among its undecided neighbours, and its
    neighbours leave (Luby rounds with a fixed priority). Links of any state
    count as adjacency. Returns a bool mask [V]."""
    V = row_ptr.size - 1
    nb = distinct_neighbors(row_ptr, col).astype(np.int64)
    owner = np.repeat(np.arange(V), np.diff(row_ptr.astype(np.int64)))
    colv = col.astype(np.int64)
    real = colv != owner
    owner, colv = owner[real], colv[real]
    prio = nb * V + np.arange(V)
    state = np.where(nb <= max_nbrs, 0, 2)  # 0 undecided, 1 leaf, 2 excluded
    big = np.iinfo(np.int64).max
    while np.any(state == 0):
        und = state == 0
        m = und[owner] & und[colv]
        nbmin = np.full(V, big, np.int64)
        np.minimum.at(nbmin, owner[m], prio[colv[m]])
        join = und & (prio < nbmin)
        state[join] = 1
        state[colv[join[owner]]] = np.where(state[colv[join[owner]]] == 1, 1, 2)
    leaf = state == 1
    assert not np.any(leaf[owner] & leaf[colv]), "leaf set is not independent"
    return leaf


def wderive_plan(roots: np.ndarray, leaf: np.ndarray, row_ptr: np.ndarray, col: np.ndarray):
    """Split a rank's roots into (cover roots run by the per-root kernel, leaf
    roots derived): the cover set is the roots not in `leaf` plus every
    neighbour of a derived leaf root (their rows feed the derivation), sorted
    and unique; the leaf roots keep their order."""
    roots = np.asarray(roots, np.uint32)
    lr = roots[leaf[roots]]
    cover = np.union1d(roots[~leaf[roots]], closure(lr, row_ptr, col))
    cover = cover[~leaf[cover]] if lr.size else cover
    return cover.astype(np.uint32), lr
