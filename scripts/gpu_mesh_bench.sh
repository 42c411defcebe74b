set -o pipefail
mkdir -p gpurun_out
for B in 1024; do
timeout -k 10 600 python -u bench.py --topology mesh1m --batch $B --steps 2 --warmup 1 --no-cpu --iso-reps 1 > gpurun_out/s22_mesh_b$B.json 2> gpurun_out/s22_mesh_b$B.err || { echo MESH_FAIL; tail -20 gpurun_out/s22_mesh_b$B.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/s22_mesh_b$B.json'));print($B, d['value'], d['gteps'], d['ms_per_step'])"
done
