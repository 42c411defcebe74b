set -o pipefail
T=${TAG:-r2s40}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pf -o run --output-format csv -- python3 scripts/exp_derive.py --reps 0 --check 0 > $O/pf.log 2>&1 || { echo PF_FAIL; tail -5 $O/pf.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pw -o run --output-format csv -- python3 scripts/exp_derive.py --reps 0 --check 0 > $O/pw.log 2>&1 || { echo PW_FAIL; tail -5 $O/pw.log; exit 1; }
python3 scripts/pmc_by_kernel.py $O/pf $O/pw > $O/pmc_by_kernel.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 scripts/exp_derive.py --reps 1 --check 0 > $O/kt.log 2>&1 || { echo KT_FAIL; tail -5 $O/kt.log; exit 1; }
python3 - <<PY
import json
d=json.load(open('$O/pmc_by_kernel.json'))
for k,v in d.items(): print(k, round(v.get('FETCH_SIZE',0)*2/1e6,2), 'GB fetch(x2)', round(v.get('WRITE_SIZE',0)/1e6,2), 'GB write', v['dispatches'])
PY
