set -o pipefail
O=gpurun_out/r2s45
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_wderive.py > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "Error|assert|FAIL" $O/pytest.log | head -30; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
