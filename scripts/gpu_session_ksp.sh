set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "ksp2 or kth or msbfs" > gpurun_out/s17_pytest_ksp.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/s17_pytest_ksp.log; exit 1; }
tail -2 gpurun_out/s17_pytest_ksp.log
timeout -k 10 400 python -u scripts/bench_ksp2.py --steps 3 > gpurun_out/s17_ksp.json 2> gpurun_out/s17_ksp.err || { echo BIG_FAIL; tail -20 gpurun_out/s17_ksp.err; exit 1; }
cat gpurun_out/s17_ksp.json
