# Round-end confirmation: smoke(), incremental and KSP2 benches on the final build.
set -o pipefail
T=${TAG:-s32}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/$T/smoke.log; exit 1; }
tail -1 gpurun_out/$T/smoke.log
timeout -k 10 600 python -u scripts/bench_incremental.py > gpurun_out/$T/inc.jsonl 2> gpurun_out/$T/inc.err || { echo INC_FAIL; tail -20 gpurun_out/$T/inc.err; exit 1; }
cut -c1-300 gpurun_out/$T/inc.jsonl
timeout -k 10 400 python -u scripts/bench_ksp2.py --steps 3 > gpurun_out/$T/ksp.json 2> gpurun_out/$T/ksp.err || { echo KSP_FAIL; tail -20 gpurun_out/$T/ksp.err; exit 1; }
cut -c1-300 gpurun_out/$T/ksp.json
