"""CPU: the C-ABI libraries load and export every function include/*.h declares."""
import ctypes
import os
import re

import pytest

from openr_amd import _native as N
from openr_amd.build import DECISION_SO, ENGINE_SO

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared(header):
    txt = open(os.path.join(ROOT, "include", header)).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b((?:ospf|odl)_[a-z0-9_]+)\s*\(", txt)))


@pytest.mark.parametrize("header,so", [("openr_spf.h", ENGINE_SO),
                                       ("openr_decision.h", DECISION_SO)])
def test_exports_every_declared_symbol(header, so):
    names = declared(header)
    assert len(names) >= 10
    lib = ctypes.CDLL(so)
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_binding_lists_match_headers():
    assert sorted(N.ENGINE_SYMBOLS) == declared("openr_spf.h")
    assert sorted(N.DECISION_SYMBOLS) == declared("openr_decision.h")


def test_engine_library_is_gfx950():
    out = os.popen(f"/opt/rocm/lib/llvm/bin/clang-offload-bundler --list --type=o "
                   f"--input={ENGINE_SO} 2>/dev/null").read()
    if not out:  # bundler cannot read .so directly on some builds; check the string table
        data = open(ENGINE_SO, "rb").read()
        assert b"gfx950" in data
    else:
        assert "gfx950" in out


def test_no_device_is_an_error_not_a_host_fallback():
    """Degrading to the host path is for device errors of an engine that ran
    (SURVEY.md §5); a LinkState on a box with no GPU must fail loudly, even
    with degrading on, so no result can silently come from the CPU."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from graphs import random_stream
    from openr_amd.linkstate import LinkState, LinkStateError
    st, names = random_stream(1)
    p = LinkState()
    p.set_degrade(True)
    p.apply(st)
    with pytest.raises(LinkStateError):
        p.spf_text(names[0])
    assert p.counters()["engine_degraded"] == 0
