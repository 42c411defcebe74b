set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/s23_pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/s23_pytest.log; exit 1; }
tail -2 gpurun_out/s23_pytest.log
