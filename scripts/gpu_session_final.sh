# Round-end headline: the driver's default bench command, then a rocprofv3
# kernel-trace summary of the same command.
set -o pipefail
T=${TAG:-s37}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/$T/bench.err; exit 1; }
cut -c1-300 gpurun_out/$T/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/prof -o run --output-format csv -- python3 bench.py > gpurun_out/$T/prof_bench.json 2> gpurun_out/$T/prof.err || { echo PROF_FAIL; tail -20 gpurun_out/$T/prof.err; exit 1; }
cut -d, -f1-4 gpurun_out/$T/prof/run_kernel_stats.csv | cut -c1-160 | head -12
