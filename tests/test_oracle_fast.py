"""The CSR-Dijkstra restatement (oracle fast_digests, the at-scale checker
for weighted graphs and the second CPU line) against the reference-shaped
restatement (oracle digests, itself pinned by the reference's fixtures):
identical digests on random graphs with parallel, down and overloaded links,
weighted and unit, link-metric and hop-count mode, and on the generators."""
import numpy as np
import pytest

from graphs import random_stream
from oracle import Oracle
from openr_amd import topology as T


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("wmax", [1, 20, 100000])
def test_fast_matches_reference_shaped_random(seed, wmax):
    st, names = random_stream(700 + seed, n=70, p=0.08, wmax=max(wmax, 1), unit=wmax == 1)
    o = Oracle(st)
    roots = names + ["not-a-node"]
    for metric in (True, False):
        assert np.array_equal(o.fast_digests(roots, metric, threads=4),
                              o.digests(roots, metric, threads=4))


@pytest.mark.parametrize("stream", [
    lambda: T.grid(12, weighted_seed=5),
    lambda: T.fabric(pods=10, planes=4, weighted_seed=7, max_metric=1000),
    lambda: T.fabric(pods=6, planes=4, reference_quirk=True),
    lambda: T.mesh(2000, seed=3),
], ids=["grid_w", "fabric_w1000", "fabric_quirk", "mesh2k"])
def test_fast_matches_reference_shaped_generators(stream):
    st = stream()
    o = Oracle(st)
    from openr_amd.linkstate import LinkState
    names = LinkState(stream=st).node_names()
    roots = names[:: max(1, len(names) // 40)]
    assert np.array_equal(o.fast_digests(roots, threads=4), o.digests(roots, threads=4))


@pytest.mark.parametrize("seed", range(4))
def test_threaded_ksp2_matches_serial(seed):
    """The KSP2 bench's multi-threaded CPU baseline (orc_ksp2_text_threads)
    gives the reference-shaped getKthPaths(src, d, 2) text of the serial
    restatement for every destination."""
    from graphs import random_stream
    st, names = random_stream(300 + seed, n=30, p=0.25)
    o, o2 = Oracle(st), Oracle(st)
    for src in names[:4]:
        assert o2.ksp2_text(src, names, threads=4) == o.ksp2_text(src, names)
