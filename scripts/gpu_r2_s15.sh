set -o pipefail
T=${TAG:-r2s15}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_routes.py tests/test_gpu_parity.py -k "route or reference_fixture" > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -60 $O/pytest.log; exit 1; }
tail -5 $O/pytest.log
