# Round-2 session 5: variant 7 knob sweep + per-class kernel stats / PMC.
set -o pipefail
T=${TAG:-r2s5}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "wdial or metric_above_63" > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $O/pytest.log | head -30; exit 1; }
timeout -k 10 600 python -u scripts/exp_wdial.py --topology fabric100k-w --roots 4096 --envs "" "OSPF_WD_WAVES_PER_CU=8" "OSPF_WD_WAVES_PER_CU=4" "OSPF_WD_WAVES_PER_CU=32" > $O/exp_w.jsonl 2> $O/exp_w.err || { echo EXPW_FAIL; tail -20 $O/exp_w.err; exit 1; }
cat $O/exp_w.jsonl
timeout -k 10 600 python -u scripts/exp_wdial.py --topology mesh1m --roots 2048 --W 1 --reps 1 --envs "" "OSPF_WD_WAVES_PER_CU=4" "OSPF_WD_WAVES_PER_CU=1" > $O/exp_m.jsonl 2> $O/exp_m.err || { echo EXPM_FAIL; tail -20 $O/exp_m.err; exit 1; }
cat $O/exp_m.jsonl
for P in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_VALU" "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d $O/pmc_w$i -o run --output-format csv -- python3 scripts/exp_wdial.py --topology fabric100k-w --roots 4096 --W 1 --reps 0 > $O/pmc_w$i.log 2>&1 || { echo PMC_FAIL $i; tail -5 $O/pmc_w$i.log; exit 1; }
done
echo pmc done
