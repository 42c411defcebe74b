"""CPU, world_size 2 (gloo): the multi-GPU sharding/gather path of bench.py.

Each rank computes the digests of its shard of every step (here with the CPU
oracle standing in for the engine), the records are all-gathered exactly as
bench.py does over RCCL, and rank 0 checks that the gathered records equal
the digests of the union of the ranks' roots and that the shards are disjoint.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from openr_amd import shard
from openr_amd import topology as T


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, result_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import Oracle
    from openr_amd.linkstate import LinkState
    st = T.fabric(pods=6, planes=4)
    ls = LinkState(stream=st)
    csr = ls.csr()
    names = ls.node_names()
    o = Oracle(st)
    caps = shard.neighbor_caps(shard.distinct_neighbors(csr["row_ptr"], csr["col"]))
    perm = np.random.default_rng(0x5EED).permutation(len(names)).astype(np.uint32)
    classes = shard.make_classes(perm, caps, batch=40)
    ok = True
    for step in range(3):
        mine = np.concatenate([shard.step_roots(c, step, world, rank) for c in classes])
        local = torch.from_numpy(o.digests([names[i] for i in mine]).view(np.int64))
        got = shard.digests_as_u64(shard.gather_digests(local))
        ids = [torch.zeros(len(mine), dtype=torch.int64) for _ in range(world)]
        dist.all_gather(ids, torch.from_numpy(mine.astype(np.int64)))
        all_ids = torch.cat(ids).numpy()
        if rank == 0:
            want = o.digests([names[i] for i in all_ids])
            ok &= bool(np.array_equal(got, want))
            for c in classes:  # per class, ranks' shards are disjoint
                parts = [shard.step_roots(c, step, world, r) for r in range(world)]
                if c.roots.size >= world * c.per_step:
                    ok &= len(set(np.concatenate(parts).tolist())) == world * c.per_step
    if rank == 0:
        result_q.put(ok)
    dist.destroy_process_group()


def test_two_rank_digest_gather_matches_oracle():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=5) is True


def test_nh_words_matches_engine_rule():
    from openr_amd.linkstate import LinkState
    ls = LinkState(stream=T.fabric(pods=40, planes=4))
    csr = ls.csr()
    w = shard.nh_words_of(csr["row_ptr"], csr["col"])
    names = ls.node_names()
    assert w[names.index("1-0-0")] == 2      # spine: 40 pods -> 40 neighbours
    assert w[names.index("2-0-0")] == 3      # fabric sw: 36 + 48 = 84
    assert w[names.index("3-0-0")] == 1      # rack sw: 4 planes


def _ksp2_worker(rank, world, port, result_q):
    """One rank of scripts/bench_ksp2.py's split: its destination block's
    k = 1 / k = 2 paths and its LFA neighbours' digests (the CPU restatement
    stands in for ospf_ksp2_dev here), gathered to rank 0 and reassembled."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import Oracle
    from openr_amd.linkstate import LinkState
    st = T.fabric(pods=5, planes=4)
    ls = LinkState(stream=st)
    csr = ls.csr()
    names = ls.node_names()
    o = Oracle(st)
    src = names.index("2-0-0")
    rp, col = csr["row_ptr"], csr["col"]
    nbrs = np.unique(col[rp[src]:rp[src + 1]])
    dsts, lfa = shard.ksp2_shards(len(names), nbrs, world, rank)
    mine = {int(d): (o.kth_paths("2-0-0", names[d], 1), o.kth_paths("2-0-0", names[d], 2))
            for d in dsts}
    lfa_dig = {int(u): o.digests([names[u]])[0].tolist() for u in lfa}
    parts = [None] * world
    dist.all_gather_object(parts, (mine, lfa_dig))
    if rank == 0:
        recs = shard.reassemble_by_destination([p[0] for p in parts])
        lfas = shard.reassemble_by_destination([p[1] for p in parts])
        want = {d: (o.kth_paths("2-0-0", names[d], 1), o.kth_paths("2-0-0", names[d], 2))
                for d in range(len(names))}
        ok = list(recs) == list(range(len(names))) and recs == want
        ok &= sorted(lfas) == sorted(int(u) for u in nbrs)
        ok &= all(lfas[int(u)] == o.digests([names[u]])[0].tolist() for u in nbrs)
        result_q.put(bool(ok))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_ksp2_destination_sharding_reassembles(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ksp2_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=5) is True


def test_ksp2_shards_are_disjoint_and_cover():
    nb = np.arange(84) * 7
    for world in (1, 2, 4, 8):
        ds, ls_ = zip(*(shard.ksp2_shards(1001, nb, world, r) for r in range(world)))
        assert np.array_equal(np.sort(np.concatenate(ds)), np.arange(1001))
        assert np.array_equal(np.sort(np.concatenate(ls_)), nb)
    with pytest.raises(ValueError):
        shard.reassemble_by_destination([{1: "a"}, {1: "b"}])
