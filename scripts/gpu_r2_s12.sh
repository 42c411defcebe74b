# Round-2 session 12: merged multi-pass rows + didx init: parity + headline.
set -o pipefail
T=${TAG:-r2s12}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "msbfs or fabric or grid31 or wide_root or ksp2 or reference_fixture" > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $O/pytest.log | head -30; exit 1; }
timeout -k 10 500 python -u bench.py --no-cpu > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
cut -c1-1700 $O/bench.json
