"""Random link-state graphs shared by the CPU and GPU parity tests."""
import numpy as np

from openr_amd.adjdb import AdjDb, AdjDbStream, create_adjacency


def random_stream(seed, n=40, p=0.15, parallel=0.2, overload=0.1, down=0.1, wmax=20,
                  unit=False):
    rng = np.random.default_rng(seed)
    names = [f"r{int(x)}" for x in rng.permutation(10 * n)[:n]]
    adjs = {nm: [] for nm in names}
    k = 0
    for i in range(n):
        for j in range(i + 1, n):
            if rng.random() > p:
                continue
            for _ in range(2 if rng.random() < parallel else 1):
                a, b = names[i], names[j]
                ia, ib = f"{a}-{b}-{k}", f"{b}-{a}-{k}"
                k += 1
                m1 = 1 if unit else int(rng.integers(1, wmax + 1))
                m2 = 1 if unit else int(rng.integers(1, wmax + 1))
                adjs[a].append(create_adjacency(b, ia, ib, m1, overloaded=bool(rng.random() < down)))
                adjs[b].append(create_adjacency(a, ib, ia, m2))
    dbs = [AdjDb(nm, adjs[nm], i + 1, overloaded=bool(rng.random() < overload))
           for i, nm in enumerate(names)]
    return AdjDbStream.from_dbs([dbs[i] for i in rng.permutation(n)]), names


def drained_fabric(pods, planes, seed=0, drain=0.05, down=0.03, weighted_seed=None,
                   ssw_per_plane=None):
    """topology.fabric with a random share of drained (overloaded) nodes and
    of adjacencies reported overloaded (links down), seeded."""
    from openr_amd import topology as T
    from openr_amd.adjdb import AdjDbStream
    rng = np.random.default_rng(seed)
    kw = {} if ssw_per_plane is None else {"ssw_per_plane": ssw_per_plane}
    dbs = T.fabric(pods=pods, planes=planes, weighted_seed=weighted_seed, **kw).to_dbs()
    for d in dbs:
        if rng.random() < drain:
            d.overloaded = True
        for a in d.adjs:
            if rng.random() < down:
                a.overloaded = True
    return AdjDbStream.from_dbs(dbs)


def path_dbs(n):
    """A path p000 - p001 - ... of n nodes with unit metrics: n - 1 levels
    deep from either end (names sort in path order)."""
    names = [f"p{i:04d}" for i in range(n)]
    adjs = {nm: [] for nm in names}
    for i in range(n - 1):
        a, b = names[i], names[i + 1]
        adjs[a].append(create_adjacency(b, f"{a}-{b}", f"{b}-{a}", 1))
        adjs[b].append(create_adjacency(a, f"{b}-{a}", f"{a}-{b}", 1))
    return [AdjDb(nm, adjs[nm], i + 1) for i, nm in enumerate(names)]
