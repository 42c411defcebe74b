# Round-2 probe: where does the weighted (Dial, variant 6) path spend its time?
# weighted F100k per class (serial streams), rocprofv3 kernel stats + one PMC
# traffic pass, and M1M with a small root batch.
set -o pipefail
T=${TAG:-r2s1}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --topology fabric100k-w --batch 1024 --steps 1 --warmup 1 --no-cpu --serial-streams --iso-reps 1 > $O/w100k.json 2> $O/w100k.err || { echo W_FAIL; tail -20 $O/w100k.err; exit 1; }
cut -c1-1500 $O/w100k.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_w -o run --output-format csv -- python3 bench.py --topology fabric100k-w --batch 1024 --steps 1 --warmup 0 --no-cpu --serial-streams --iso-reps 0 > /dev/null 2> $O/prof_w.err || { echo PROFW_FAIL; tail -20 $O/prof_w.err; exit 1; }
cut -d, -f1-6 $O/prof_w/run_kernel_stats.csv | cut -c1-200 | head -12
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_w -o run --output-format csv -- python3 bench.py --topology fabric100k-w --batch 1024 --steps 1 --warmup 0 --no-cpu --serial-streams --iso-reps 0 > /dev/null 2> $O/pmc_w.err || { echo PMCW_FAIL; tail -20 $O/pmc_w.err; exit 1; }
timeout -k 10 400 python -u bench.py --topology mesh1m --batch 256 --steps 1 --warmup 1 --no-cpu --iso-reps 1 > $O/m1m.json 2> $O/m1m.err || { echo M_FAIL; tail -20 $O/m1m.err; exit 1; }
cut -c1-1200 $O/m1m.json
