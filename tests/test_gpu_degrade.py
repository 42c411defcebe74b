"""Device errors are survivable ("on any device error the shim
falls back ... never aborts Decision"). A device error
is forced with the engine's test hook (ospf_inject_error: the k-th engine call
fails with OSPF_E_DEVICE); odl::LinkState must record it, release the engine
and answer that call and every later one on its own host path
(LinkState::runSpfHost, product code), with text equal to the oracle's and
decision.spf_runs unchanged in meaning. The reference ends in XLOG(FATAL)
when an exception leaves the Decision fiber (Decision.cpp:240-250).

Also here: the path's fb303 counters (decision.spf_ms / ucmp_runs / ucmp_ms /
route_build_ms, LinkState.cpp:909,926,1029, SpfSolver.cpp:640-644) and the
teardown order of r05's core dump (a sweep released after its engine)."""
import gc

import numpy as np
import pytest

from graphs import random_stream
from oracle import Oracle
from openr_amd import topology as T
from openr_amd.engine import Engine
from openr_amd.linkstate import LinkState, LinkStateError

pytestmark = pytest.mark.gpu


def pair(stream):
    o, p = Oracle(), LinkState()
    p.set_degrade(True)  # the suite runs strict (conftest.py); this file tests degrading
    assert o.apply(stream) == p.apply(stream)
    return o, p


@pytest.mark.parametrize("after", [1, 2, 3, 5])
def test_spf_degrades_to_host_path(after):
    """The after-th engine call fails (1 = the graph load); every root's
    text, both metric modes, equals the oracle's; spf_runs = the oracle's."""
    st, names = random_stream(11 + after)
    o, p = pair(st)
    p.inject_engine_error(after)
    for i, r in enumerate(names):
        if i % 7 == 0:
            p.prefetch(names[i:i + 7])  # batches: a failure in the middle of one
        assert p.spf_text(r) == o.spf_text(r), r
        assert p.spf_text(r, False) == o.spf_text(r, False), r
    c = p.counters()
    assert c["engine_errors"] == 1 and c["engine_degraded"] == 1
    assert "injected" in p.last_engine_error()
    assert p.spf_runs == o.spf_runs


def test_ksp2_and_sweep_degrade():
    """The failure inside an all-sources sweep, then KSP2 and digests on the
    host path: equal to the oracle."""
    st = T.fabric(pods=6, planes=4)
    o, p = pair(st)
    names = sorted(set(d.name for d in st.to_dbs()))
    p.inject_engine_error(2)  # load ok, the sweep create fails
    assert np.array_equal(p.all_sources_digests(), o.fast_digests(names))
    dsts = names[1::9]
    assert p.ksp2_text(names[0], dsts) == o.ksp2_text(names[0], dsts)
    assert p.counters()["engine_degraded"] == 1
    # the engine back on: same answers from the device
    p.set_host_spf(False)
    assert p.counters()["engine_degraded"] == 0
    assert np.array_equal(p.digests(names), o.fast_digests(names))
    assert p.counters()["engine_errors"] == 1


def test_strict_mode_raises():
    st, names = random_stream(3)
    o, p = pair(st)
    p.set_degrade(False)
    p.inject_engine_error(1)
    with pytest.raises(LinkStateError, match="injected"):
        p.spf_text(names[0])
    assert p.counters()["engine_errors"] == 0


def test_counters():
    """decision.spf_ms per logical run, ucmp_runs / ucmp_ms, route_build_ms."""
    st, names = random_stream(21)
    o, p = pair(st)
    p.prefetch(names)
    c = p.counters()
    assert c["spf_runs"] == len(names) == c["spf_ms_samples"] and c["spf_ms_sum"] > 0
    p.ucmp(names[0], {names[5]: 2, names[9]: 3})
    p.route_db(names[0], {"10.0.0.0/24": [[names[5], "ip", "ecmp", 0, None]]})
    c = p.counters()
    assert c["ucmp_runs"] == 1 and c["ucmp_ms_sum"] >= 0
    assert c["route_build_runs"] >= 1 and c["route_build_ms_sum"] >= 0
    assert c["engine_errors"] == 0 and c["engine_degraded"] == 0


def test_sweep_released_after_its_engine():
    """r05 core dump (gpurun_out/r5_b1): a sweep dropped after eng.close()
    must not touch the freed context (ospf_close releases live sweeps first,
    spf_engine.hip ospf_close)."""
    st = T.fabric(pods=4, planes=4)
    ls = LinkState(stream=st)
    eng = Engine(0)
    eng.load(ls.csr())
    sw = eng.sweep()
    sw.run()
    eng.sync()
    eng.close()
    del sw
    gc.collect()
    # the device is still usable afterwards
    eng2 = Engine(0)
    eng2.load(ls.csr())
    sw2 = eng2.sweep()
    sw2.run()
    eng2.sync()
    sw2.close()
    eng2.close()
