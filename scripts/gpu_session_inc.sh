set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu -k "incremental or affected or repair" > gpurun_out/s25_pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/s25_pytest.log; exit 1; }
tail -2 gpurun_out/s25_pytest.log
timeout -k 10 600 python -u scripts/bench_incremental.py > gpurun_out/s25_inc.jsonl 2> gpurun_out/s25_inc.err || { echo INC_FAIL; tail -20 gpurun_out/s25_inc.err; exit 1; }
cat gpurun_out/s25_inc.jsonl; tail -3 gpurun_out/s25_inc.err
