set -o pipefail
T=${TAG:-r2s18}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_derive.py > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 600 python -u scripts/exp_derive.py > $O/derive.json 2> $O/derive.err || { echo EXP_FAIL; tail -30 $O/derive.err; exit 1; }
cat $O/derive.json
timeout -k 10 600 python -u bench.py --steps 10 --warmup 2 > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
