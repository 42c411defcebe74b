set -o pipefail
T=${TAG:-r2s23}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_derive.py > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 600 python -u bench.py --steps 10 --warmup 2 > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -30 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],[ (c.get('launch') or c.get('cap'), c.get('path'), c['isolated_launch_ms']) for c in d['config']['root_classes']], d['parity_vs_cpu_sample'])"
i=0
for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_SALU SQ_BUSY_CYCLES" \
         "FETCH_SIZE TCC_HIT_sum" "WRITE_SIZE TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P -d $O/p$i -o run --output-format csv -- python3 scripts/exp_derive.py --reps 0 --check 0 > $O/p$i.log 2>&1 || { echo PMC_FAIL $i; tail -5 $O/p$i.log; exit 1; }
done
python scripts/pmc_by_kernel.py $O/p1 $O/p2 $O/p3 > $O/pmc.json
python -c "
import json;d=json.load(open('$O/pmc.json'))
for k,v in d.items(): print(k, {c: round(v[c]/1e6,1) for c in ('FETCH_SIZE','WRITE_SIZE','SQ_WAIT_ANY','SQ_WAVE_CYCLES','SQ_INSTS_VALU') if c in v})"
