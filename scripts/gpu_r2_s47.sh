set -o pipefail
O=gpurun_out/r2s47
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wderive.py > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "Error|assert" $O/pytest.log | head; tail -20 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 600 python -u bench.py --topology fabric100k-w --steps 5 --warmup 1 > $O/bench_w.json 2> $O/bench_w.err || { echo BENCH_FAIL; tail -30 $O/bench_w.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_w.json'));print(d['value'],d['ms_per_step'],[(u['launch'],u['isolated_launch_ms'],u['frac']) for u in d['roofline']['launches']], d['config']['root_classes'], d['parity_vs_cpu_sample'])"
