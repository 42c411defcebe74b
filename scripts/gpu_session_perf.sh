# Parity, per-class timings (each class alone), the headline bench.
set -o pipefail
T=${TAG:-s40}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/$T/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/$T/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/$T/pytest_gpu.log
for c in 1:14003 3:2334 56:47; do
  timeout -k 10 300 python -u scripts/exp_class.py --W ${c%%:*} --n ${c##*:} --reps 3 >> gpurun_out/$T/cls.jsonl 2> gpurun_out/$T/cls.err || { echo CLS_FAIL; tail -20 gpurun_out/$T/cls.err; exit 1; }
done
cut -c1-200 gpurun_out/$T/cls.jsonl
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/$T/bench.err; exit 1; }
cut -c1-400 gpurun_out/$T/bench.json
