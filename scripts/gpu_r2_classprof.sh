# Per-class single-stream profiles of the headline (F100k unit, all-sources
# classes): rocprofv3 kernel stats + FETCH/WRITE passes -> profiles/<round>/.
# Usage: bash scripts/gpu_r2_classprof.sh [topology] (roots per class = all)
set -o pipefail
T=${TAG:-r2prof}
TOPO=${TOPO:-fabric100k}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
R=3
for CAP in ${CAPS:-8 96 1792}; do
  CMD="python3 bench.py --topology $TOPO --class-only $CAP --reps $R"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_$CAP -o run --output-format csv -- $CMD > $O/kt_$CAP.log 2>&1 || { echo KT_FAIL $CAP; tail -5 $O/kt_$CAP.log; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_$CAP -o run --output-format csv -- $CMD > $O/fetch_$CAP.log 2>&1 || { echo FETCH_FAIL $CAP; tail -5 $O/fetch_$CAP.log; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/write_$CAP -o run --output-format csv -- $CMD > $O/write_$CAP.log 2>&1 || { echo WRITE_FAIL $CAP; tail -5 $O/write_$CAP.log; exit 1; }
  grep -o "launches of [0-9]* roots" $O/kt_$CAP.log
  echo class $CAP ok
done
