# Per-class kernel split (rocprofv3) for the W = 3 class, then the headline bench.
set -o pipefail
T=${TAG:-s29}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/$T/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/$T/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/$T/pytest_gpu.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/prof_w3 -o run --output-format csv -- python3 scripts/exp_class.py --W 3 --n 2334 --reps 3 > gpurun_out/$T/w3.jsonl 2> gpurun_out/$T/w3.err || { echo W3_FAIL; tail -20 gpurun_out/$T/w3.err; exit 1; }
cat gpurun_out/$T/w3.jsonl
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/$T/bench.err; exit 1; }
cat gpurun_out/$T/bench.json
