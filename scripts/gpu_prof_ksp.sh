set -o pipefail
mkdir -p gpurun_out/ksp_prof
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ksp_prof -o run --output-format csv -- python3 scripts/bench_ksp2.py --steps 1 --warmup 1 --iso-reps 1 --no-cpu > gpurun_out/ksp_prof/bench.json 2> gpurun_out/ksp_prof/bench.err || { echo PROF_FAIL; tail -20 gpurun_out/ksp_prof/bench.err; exit 1; }
f=$(find gpurun_out/ksp_prof -name "*kernel_trace.csv" | head -1)
python3 scripts/ksp_dispatch.py "$f"
