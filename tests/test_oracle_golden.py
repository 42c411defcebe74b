"""CPU: the oracle restatement against the reference's own known answers
(tests/golden/*.json, transcribed from LinkStateTest.cpp / DecisionTest.cpp)."""
import pytest

from golden_eval import OracleLS, load_fixtures, run_fixture

FIXTURES = load_fixtures()


@pytest.mark.parametrize("fx", FIXTURES, ids=[f["name"] for f in FIXTURES])
def test_oracle_matches_reference_fixture(fx):
    assert run_fixture(fx, OracleLS) > 0


def test_fixture_inventory():
    names = {f["name"] for f in FIXTURES}
    for must in ("linkstate_basic_operation", "linkstate_kth_paths_box",
                 "decision_simple_ring_ksp2", "decision_parallel_adj_ring_ksp2",
                 "decision_grid_16", "decision_overload_node"):
        assert must in names
