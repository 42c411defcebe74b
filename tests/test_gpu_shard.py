"""KSP2 destinations and root batches split across the device slots of a
multi-device odl::LinkState (VERDICT r04 missing #2, SURVEY §8(e): "for KSP2,
shard the destinations of one root"; the LFA-style batch of a root's
neighbours' runSpf). Two slots on device 0 (two engine
contexts on one card, each with its own streams and scratch) against the
single-slot LinkState and the oracle: the same records, the same spf_runs.
Reference: LinkState::getKthPaths (openr/decision/LinkState.cpp:790-819),
SpfSolver's KSP2 route build (openr/decision/SpfSolver.cpp:847-973)."""
import numpy as np
import pytest

from graphs import random_stream
from link_events import both
from oracle import Oracle
from openr_amd import topology as T
from openr_amd.linkstate import LinkState

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("slots", [2, 3])
@pytest.mark.parametrize("seed", range(3))
def test_ksp2_destinations_split_across_slots(seed, slots):
    st, names = random_stream(700 + seed, n=60, unit=bool(seed & 1))
    o, p = both(st)
    q = LinkState(devices=[0] * slots)
    q.apply(st)
    for src in names[:4]:
        want = o.ksp2_text(src, names)
        assert p.ksp2_text(src, names) == want, src
        assert q.ksp2_text(src, names) == want, src
    assert q.spf_runs == p.spf_runs == o.spf_runs
    ss = q.shard_stats()
    assert ss["ksp2_runs"] == 4 and ss["ksp2_launches"] == 4 * slots


def test_fabric_ksp2_all_destinations_two_slots():
    """BASELINE config 4's shape (KSP2 from FSW "2-0-0" to every node),
    small, on two slots."""
    st = T.fabric(pods=8, planes=4)
    o = Oracle(st)
    q = LinkState(devices=[0, 0], stream=st)
    dsts = q.node_names()
    assert q.ksp2_text("2-0-0", dsts) == o.ksp2_text("2-0-0", dsts)
    assert q.spf_runs == o.spf_runs
    assert q.shard_stats()["ksp2_launches"] == 2


@pytest.mark.parametrize("unit", [True, False])
def test_neighbour_batches_split_across_slots(unit):
    """A root's neighbours' runSpf as one prefetch (the LFA-style batch):
    rows split across the slots, every result equal to the single slot's and
    the oracle's."""
    st, names = random_stream(730, n=80, unit=unit)
    o = Oracle(st)
    q = LinkState(devices=[0, 0], stream=st)
    rng = np.random.default_rng(3)
    roots = rng.choice(names, 24, replace=False).tolist()
    q.prefetch(roots)
    q.prefetch(roots, False)
    for r in roots:
        assert q.spf_text(r) == o.spf_text(r), r
        assert q.spf_text(r, False) == o.spf_text(r, False), r
    ss = q.shard_stats()
    assert ss["spf_batches"] >= 2 and ss["spf_launches"] == 2 * ss["spf_batches"]
    assert q.spf_runs == 48
