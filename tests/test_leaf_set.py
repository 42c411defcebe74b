"""Leaf-set selection for the weighted derive (CPU): independence, the
neighbour bound, maximality, and the fabric's racks."""
import numpy as np

from graphs import random_stream
from openr_amd import shard
from openr_amd import topology as T
from openr_amd.linkstate import LinkState


def _csr(stream):
    ls = LinkState()
    ls.apply(stream)
    return ls, ls.csr()


def test_leaf_set_random_graphs_independent_and_maximal():
    for seed in range(5):
        _, csr = _csr(random_stream(seed, n=120, p=0.05)[0])
        rp, col = csr["row_ptr"], csr["col"]
        V = rp.size - 1
        leaf = shard.leaf_set(rp, col, max_nbrs=6)
        nb = shard.distinct_neighbors(rp, col)
        owner = np.repeat(np.arange(V), np.diff(rp.astype(np.int64)))
        real = col != owner
        assert not np.any(leaf[owner[real]] & leaf[col[real]])
        assert np.all(nb[leaf] <= 6)
        # maximal: every candidate outside the set has a leaf neighbour
        has_leaf_nb = np.zeros(V, bool)
        has_leaf_nb[owner[real][leaf[col[real]]]] = True
        assert np.all(leaf | (nb > 6) | has_leaf_nb)


def test_leaf_set_fabric_is_the_racks():
    """Racks (8 fabric switches each) always; spines too while they have at
    most 32 neighbours (pods); fabric switches (48 racks + 36 spines) never."""
    ls, csr = _csr(T.fabric(pods=40, planes=8, weighted_seed=7))
    names = ls.node_names()
    leaf = shard.leaf_set(csr["row_ptr"], csr["col"])
    assert {names[i] for i in np.nonzero(leaf)[0]} == {n for n in names if n.startswith("3-")}
    ls, csr = _csr(T.fabric(pods=20, planes=8, weighted_seed=7))
    names = ls.node_names()
    leaf = shard.leaf_set(csr["row_ptr"], csr["col"])
    assert {names[i] for i in np.nonzero(leaf)[0]} == {n for n in names if n[0] in "13"}
    cover, lr = shard.wderive_plan(np.arange(len(names)), leaf, csr["row_ptr"], csr["col"])
    assert cover.size + lr.size == len(names)
    # a rank owning pods 0..4: its cover = its fabric switches only
    mine = np.array([i for i, n in enumerate(names) if n[0] in "23" and int(n.split("-")[1]) < 5],
                    np.uint32)
    cover, lr = shard.wderive_plan(mine, leaf, csr["row_ptr"], csr["col"])
    assert {names[i][0] for i in cover} == {"2"} and cover.size == 5 * 8
    assert lr.size == 5 * 48
    # a rank owning spines of plane 0: its cover adds plane 0's fabric switches
    sp = np.array([names.index(f"1-0-{i}") for i in range(3)], np.uint32)
    cover, lr = shard.wderive_plan(sp, leaf, csr["row_ptr"], csr["col"])
    assert sorted(names[i] for i in cover) == sorted(f"2-{d}-0" for d in range(20))
