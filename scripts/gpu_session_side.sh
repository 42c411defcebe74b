# Side benches (SURVEY.md §8 rows beyond the headline): incremental updates,
# KSP2 + LFA (config 4), weighted 1M mesh (config 5). Stops at the first failure.
set -o pipefail
T=${TAG:-s25}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 600 python -u scripts/bench_incremental.py > gpurun_out/$T/inc.jsonl 2> gpurun_out/$T/inc.err || { echo INC_FAIL; tail -20 gpurun_out/$T/inc.err; exit 1; }
cat gpurun_out/$T/inc.jsonl
timeout -k 10 400 python -u scripts/bench_ksp2.py --steps 3 > gpurun_out/$T/ksp.json 2> gpurun_out/$T/ksp.err || { echo KSP_FAIL; tail -20 gpurun_out/$T/ksp.err; exit 1; }
cat gpurun_out/$T/ksp.json
timeout -k 10 600 python -u bench.py --topology mesh1m --batch 1024 --steps 2 --warmup 1 --no-cpu --iso-reps 1 > gpurun_out/$T/mesh.json 2> gpurun_out/$T/mesh.err || { echo MESH_FAIL; tail -20 gpurun_out/$T/mesh.err; exit 1; }
cat gpurun_out/$T/mesh.json
