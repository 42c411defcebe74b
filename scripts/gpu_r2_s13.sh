set -o pipefail
T=${TAG:-r2s13}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for CAP in 96 1792; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_$CAP -o run --output-format csv -- python3 bench.py --class-only $CAP --reps 3 > $O/kt_$CAP.log 2>&1 || { echo KT_FAIL; tail -5 $O/kt_$CAP.log; exit 1; }
cut -d, -f1-4 $O/kt_$CAP/run_kernel_stats.csv | cut -c1-150 | head -9
done
