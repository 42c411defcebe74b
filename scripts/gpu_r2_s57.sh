set -o pipefail
O=gpurun_out/r2s57
mkdir -p $O
export TMPDIR=/tmp
START=$(date +%s)
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -30 $O/bench.err; exit 1; }
echo "wall $(( $(date +%s) - START )) s"
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],d['steps'],d['roofline']['frac'],d['roofline']['step_frac'],d['parity_vs_cpu_sample'])"
