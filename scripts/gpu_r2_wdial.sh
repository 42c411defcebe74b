# Round-2: variant 7 (wave-per-root Dial) parity + first weighted numbers.
set -o pipefail
T=${TAG:-r2s3}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "wdial or metric_above_63 or mesh_60k or fabric_sampled" > $O/pytest.log 2>&1; rc=$?
tail -5 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $O/pytest.log | head -30; exit 1; }
timeout -k 10 300 python -u bench.py --topology fabric100k-w --batch 4096 --steps 2 --warmup 1 --no-cpu --serial-streams --iso-reps 1 > $O/w100k.json 2> $O/w100k.err || { echo W_FAIL; tail -20 $O/w100k.err; exit 1; }
cut -c1-1500 $O/w100k.json
timeout -k 10 400 python -u bench.py --topology mesh1m --batch 2048 --steps 1 --warmup 1 --no-cpu --iso-reps 1 > $O/m1m.json 2> $O/m1m.err || { echo M_FAIL; tail -20 $O/m1m.err; exit 1; }
cut -c1-1200 $O/m1m.json
