set -o pipefail
T=${TAG:-r2s16}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1500 python -u -m pytest -x -v -s --timeout 900 --timeout-method thread tests/test_gpu_multirank.py tests/test_gpu_scale.py tests/test_out_of_contract.py "tests/test_gpu_parity.py::test_out_of_contract_update_switches_to_host_and_back" "tests/test_gpu_parity.py::test_ksp2_ignore_set_above_run_list_cap" > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -80 $O/pytest.log; exit 1; }
tail -15 $O/pytest.log
timeout -k 10 600 python -u scripts/prod_callstack.py > $O/prod_callstack.json 2> $O/prod_callstack.err || { echo PROD_FAIL; tail -30 $O/prod_callstack.err; exit 1; }
cat $O/prod_callstack.json
