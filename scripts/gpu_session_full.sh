set -o pipefail
mkdir -p gpurun_out
T=${TAG:-s28}
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/${T}_pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
timeout -k 10 600 python -u scripts/bench_incremental.py > gpurun_out/${T}_inc.jsonl 2> gpurun_out/${T}_inc.err || { echo INC_FAIL; tail -20 gpurun_out/${T}_inc.err; exit 1; }
cat gpurun_out/${T}_inc.jsonl; tail -3 gpurun_out/${T}_inc.err
