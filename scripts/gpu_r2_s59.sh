set -o pipefail
O=gpurun_out/r2s59
mkdir -p $O
export TMPDIR=/tmp
for env in "OPENR_DERIVE_SERIAL=0" "OPENR_DERIVE_SERIAL=1" "OPENR_DERIVE_SERIAL=0" "OPENR_DERIVE_SERIAL=1"; do
  env $env timeout -k 10 400 python -u bench.py --steps 30 --warmup 2 --no-cpu --iso-reps 1 > $O/b.json 2> $O/b.err || { echo BENCH_FAIL; tail -30 $O/b.err; exit 1; }
  python -c "import json;d=json.load(open('$O/b.json'));print('$env', d['value'],d['ms_per_step'])"
done
