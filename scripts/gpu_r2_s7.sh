# Round-2 session 7: packed variant 7 + neighbour-capacity classes.
set -o pipefail
T=${TAG:-r2s10}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "wdial or metric_above_63" > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $O/pytest.log | head -30; exit 1; }
timeout -k 10 600 python -u scripts/exp_wdial.py --topology fabric100k-w --roots 16384 --envs "" "OSPF_WD_GROUP=8" > $O/exp_w.jsonl 2> $O/exp_w.err || { echo EXPW_FAIL; tail -20 $O/exp_w.err; exit 1; }
cat $O/exp_w.jsonl
timeout -k 10 600 python -u scripts/exp_wdial.py --topology mesh1m --roots 4096 --reps 1 --envs "" "OSPF_WD_GROUP=2" "OSPF_WD_GROUP=4" > $O/exp_m.jsonl 2> $O/exp_m.err || { echo EXPM_FAIL; tail -20 $O/exp_m.err; exit 1; }
cat $O/exp_m.jsonl
