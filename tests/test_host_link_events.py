"""The link-event sequences of tests/test_gpu_link_events.py run GPU-free:
odl::LinkState with every SPF / KSP2 / digest on the host
(odl_set_host_spf; runSpfHost is the reference's algorithm,
openr/decision/LinkState.cpp:836-911), so the ingest, the in-place CSR
splice (patchStructure, [LINK UP] / [LINK DOWN] LinkState.cpp:632-657), the
memo drop and its background release (clearMemo, :751-754) and decision.spf_runs
are checked against the oracle in the container -- and can run against
sanitizer builds of libopenr_decision.so / liboracle.so
(scripts/sanitize_host.sh)."""
import pytest

import link_events as LE
from link_events import both
from graphs import random_stream


@pytest.mark.parametrize("seed", range(4))
@pytest.mark.parametrize("unit", [False, True])
def test_link_down_up_random_graphs_host(seed, unit):
    LE.link_down_up_random_graphs(seed, unit, host=True)


def test_link_events_mixed_with_metric_and_overload_host():
    LE.link_events_mixed_with_metric_and_overload(host=True)


def test_parallel_link_ranks_after_insert_host():
    LE.parallel_link_ranks_after_insert(host=True)


def test_host_spf_switch_never_opens_the_engine():
    """With host SPF on, no device load and no sweep happen, whatever is asked."""
    st, names = random_stream(5, n=30)
    o, p = both(st, host=True)
    for r in names[:5]:
        assert p.spf_text(r) == o.spf_text(r)
        assert p.spf_text(r, False) == o.spf_text(r, False)
    p.prefetch_all()
    p.prefetch(names)
    p.ksp2_text(names[0], names[1:6])
    assert p.topology_stats()["loads"] == 0
    assert p.sweep_stats()["sweeps"] == 0


@pytest.mark.parametrize("seed", range(3))
@pytest.mark.parametrize("unit", [False, True])
def test_node_remove_add_in_place_host(seed, unit):
    LE.node_remove_add_random_graphs(seed, unit, host=True)
