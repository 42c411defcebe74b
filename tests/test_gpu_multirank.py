"""bench.py's multi-GPU path, rehearsed with two ranks on one GPU: the real
step code (ospf_sweep_run over the rank's part of the library's root
partition), the all-gather of the timed step's digests, max-over-ranks
timing, and rank 0's check of the gathered digests against the CPU
restatement. Collectives run on gloo here (RCCL will not put two ranks on
one device); RCCL itself is exercised only by the driver's 8-GPU runs. The
ranks are launched by tests/conftest.py before this process touches the GPU."""
import json

import pytest

from conftest import MULTIRANK

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(600)
@pytest.mark.parametrize("kind,mode", [("unit", "derive"), ("weighted", "wcover")])
def test_two_rank_bench_step_and_gather(kind, mode):
    run = MULTIRANK[kind]
    proc = run["proc"]
    rc = proc.wait(timeout=540)
    err = open(run["err"]).read()
    assert rc == 0, err[-4000:]
    lines = [json.loads(x) for x in open(run["out"]).read().splitlines()
             if x.startswith("{")]
    assert len(lines) == 1, lines  # rank 0 prints the one line
    ln = lines[0]
    assert ln["n_gpus"] == 2 and ln["steps"] == 2 and ln["dist_backend"] == "gloo"
    assert ln["gathered_roots"] == ln["config"]["n_nodes"]  # every root once
    assert ln["parity_vs_cpu_sample"]["roots"] == 96
    assert ln["parity_vs_cpu_sample"]["equal"] is True
    assert ln["value"] > 0 and ln["config"]["roots_per_step"] == ln["config"]["n_nodes"]
    assert ln["config"]["mode"] == "sweep:" + mode  # the library's sweep, one call per step
