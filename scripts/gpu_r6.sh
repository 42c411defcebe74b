#!/bin/bash
# Round-6 GPU session driver. Steps (space-separated in STEPS):
#   sweep   pytest tests/test_gpu_sweep.py
#   gpu     the whole -m gpu suite
#   scale   tests/test_gpu_scale.py only
#   scale4  tests/test_gpu_scale_sweeps.py (full-size sweeps with drains / weights)
#   t       pytest $TESTS;  script  python $SCRIPT
#   bench   python bench.py (default headline config)
#   benchT  python bench.py --topology $TOPO
#   prof    rocprofv3 --kernel-trace --stats of a short bench
# Each GPU step has its own time limit; the first failure ends the call.
set -u
TAG=${1:-s}; OUT=gpurun_out/r6_$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
STEPS=${STEPS:-"sweep bench"}
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
for st in $STEPS; do
  case $st in
    sweep) timeout -k 10 600 $PYT tests/test_gpu_sweep.py > "$OUT/sweep.log" 2>&1; rc=$?
           tail -5 "$OUT/sweep.log";;
    gpu)   timeout -k 10 1000 $PYT -q -m gpu tests > "$OUT/gpu.log" 2>&1; rc=$?
           tail -5 "$OUT/gpu.log";;
    scale) timeout -k 10 900 $PYT -s tests/test_gpu_scale.py ${SCALE_K:+-k "$SCALE_K"} > "$OUT/scale.log" 2>&1; rc=$?
           tail -8 "$OUT/scale.log";;
    bench) timeout -k 10 420 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"; rc=$?
           cat "$OUT/bench.json"; tail -3 "$OUT/bench.err";;
    benchT) timeout -k 10 600 python bench.py --topology $TOPO ${BENCH_ARGS:-} > "$OUT/bench_$TOPO.json" 2> "$OUT/bench_$TOPO.err"; rc=$?
           cat "$OUT/bench_$TOPO.json"; tail -3 "$OUT/bench_$TOPO.err";;
    prof)  timeout -k 10 420 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
             python bench.py --steps 5 --warmup 1 --no-cpu ${PROF_ARGS:-} > "$OUT/prof_bench.json" 2> "$OUT/prof.err"; rc=$?
           tail -3 "$OUT/prof.err";;
    csv)   timeout -k 10 420 rocprofv3 --kernel-trace --stats -d "$OUT/csv" -o run --output-format csv -- \
             python bench.py --steps 5 --warmup 1 --no-cpu ${PROF_ARGS:-} > "$OUT/csv_bench.json" 2> "$OUT/csv.err"; rc=$?
           tail -2 "$OUT/csv.err";;
    pmc)   rc=0; i=0
           for P in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"; do
             i=$((i+1))
             timeout -s KILL 120 rocprofv3 --pmc $P -d "$OUT/pmc$i" -o run --output-format csv -- \
               python bench.py --steps 1 --warmup 0 --no-cpu --iso-reps 1 ${PROF_ARGS:-} > "$OUT/pmc$i.log" 2>&1; rc=$?
             echo "pmc pass $i rc=$rc"; [ $rc -eq 0 ] || break
           done
           [ $rc -eq 0 ] && python scripts/pmc_by_kernel.py "$OUT"/pmc* > "$OUT/pmc_by_kernel.json";;
    unitprof)  # per-launch-unit kernel time + HBM traffic of the sweep (scripts/sweep_unit_stats.py)
           timeout -k 10 420 rocprofv3 --kernel-trace --stats -d "$OUT/utrace" -o run --output-format csv -- \
             python bench.py --steps 5 --warmup 1 --no-cpu --iso-reps 3 ${PROF_ARGS:-} > "$OUT/utrace_bench.json" 2> "$OUT/utrace.err"; rc=$?
           [ $rc -eq 0 ] && OSPF_LV_SERIAL=1 timeout -k 10 420 rocprofv3 --kernel-trace --stats -d "$OUT/utrace_serial" -o run --output-format csv -- \
             python bench.py --steps 2 --warmup 1 --no-cpu --iso-reps 3 ${PROF_ARGS:-} > "$OUT/utrace_serial_bench.json" 2>> "$OUT/utrace.err"; rc=$?
           i=0
           for P in FETCH_SIZE WRITE_SIZE; do
             [ $rc -eq 0 ] || break
             i=$((i+1))
             timeout -s KILL 180 rocprofv3 --pmc $P -d "$OUT/upmc$i" -o run --output-format csv -- \
               python bench.py --steps 1 --warmup 0 --no-cpu --iso-reps 1 ${PROF_ARGS:-} > "$OUT/upmc$i.json" 2> "$OUT/upmc$i.err"; rc=$?
             echo "pmc pass $P rc=$rc"
           done
           if [ $rc -eq 0 ]; then
             python scripts/sweep_unit_stats.py --bench "$OUT/utrace_bench.json" --trace "$OUT/utrace" --reps 3 --out "$OUT/units_trace.json" &&
             python scripts/sweep_unit_stats.py --bench "$OUT/utrace_serial_bench.json" --trace "$OUT/utrace_serial" --reps 3 --out "$OUT/units_trace_serial.json" &&
             python scripts/sweep_unit_stats.py --bench "$OUT/upmc1.json" --pmc "$OUT/upmc1" "$OUT/upmc2" --reps 1 --out "$OUT/pmc_traffic.json"; rc=$?
           fi;;
    upmcsq)  # per-unit SQ counters (instructions, busy / wait cycles) of the sweep
           timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY -d "$OUT/upmcsq" -o run --output-format csv -- \
             python bench.py --steps 1 --warmup 0 --no-cpu --iso-reps 1 ${PROF_ARGS:-} > "$OUT/upmcsq.json" 2> "$OUT/upmcsq.err"; rc=$?
           [ $rc -eq 0 ] && python scripts/sweep_unit_stats.py --bench "$OUT/upmcsq.json" --pmc "$OUT/upmcsq" --reps 1 --out "$OUT/pmc_sq.json" > /dev/null; rc=$?;;
    ab)    # A/B of env knobs on the default bench: AB="NAME=1 OTHER=1 ..." (one run each + baseline)
           rc=0
           for kv in base ${AB:-}; do
             if [ "$kv" = base ]; then E=""; else E="${kv//,/ }"; fi
             timeout -k 10 300 env $E python bench.py --steps 20 --warmup 2 --cpu-sample 8 --iso-reps 2 ${AB_ARGS:-} > "$OUT/ab_$kv.json" 2> "$OUT/ab_$kv.err"; rc=$?
             echo "ab $kv rc=$rc $(python -c "import json,sys; d=json.load(open('$OUT/ab_$kv.json')); print(d['value'], d['ms_per_step'], d['parity_vs_cpu_sample'])" 2>/dev/null)"
             [ $rc -eq 0 ] || break
           done;;
    debug) timeout -k 10 300 python scripts/debug/${DBG:-stage_digests.py} > "$OUT/debug.log" 2>&1; rc=$?
           tail -30 "$OUT/debug.log";;
    scale4) timeout -k 10 1100 $PYT -s tests/test_gpu_scale_sweeps.py ${SCALE_K:+-k "$SCALE_K"} > "$OUT/scale4.log" 2>&1; rc=$?
           tail -8 "$OUT/scale4.log";;
    ksp)   timeout -k 10 ${K_LIMIT:-600} python -u scripts/bench_ksp2.py ${KSP_ARGS:-} > "$OUT/ksp2.json" 2> "$OUT/ksp2.err"; rc=$?
           tail -c 1500 "$OUT/ksp2.json"; tail -3 "$OUT/ksp2.err";;
    t)     timeout -k 10 ${T_LIMIT:-600} $PYT -s $TESTS > "$OUT/t.log" 2>&1; rc=$?
           tail -8 "$OUT/t.log";;
    script) timeout -k 10 ${S_LIMIT:-600} python -u $SCRIPT > "$OUT/script.out" 2> "$OUT/script.err"; rc=$?
           tail -5 "$OUT/script.out"; tail -5 "$OUT/script.err";;
    derive) timeout -k 10 600 $PYT tests/test_gpu_derive.py tests/test_gpu_wderive.py > "$OUT/derive.log" 2>&1; rc=$?
           tail -3 "$OUT/derive.log";;
    records)  # all-sources throughput without fabric symmetry (no twins to derive from)
           rc=0
           for spec in "grid100:" "grid31:" "fabric100k:OSPF_SWEEP_NOTWIN=1,OSPF_SWEEP_NOTWINLV=1" "fabric100k-w:OSPF_SEED_NONH=1,OSPF_CLOSURE_NONH=1"; do
             T=${spec%%:*}; E=${spec#*:}; E=${E//,/ }; tag=${T}${E:+_ab}
             timeout -k 10 420 env $E python bench.py --topology $T --steps 10 --warmup 2 --cpu-sample 8 > "$OUT/rec_$tag.json" 2> "$OUT/rec_$tag.err"; rc=$?
             echo "record $tag rc=$rc $(head -c 300 "$OUT/rec_$tag.json")"
             [ $rc -eq 0 ] || break
           done;;
    m1m)   # M1M: multi-root sweep part (wmulti) vs the per-root Dial batch (+ in-flight knob)
           rc=0
           for spec in "wmulti:--mode wmulti" ${M1M_EXTRA:-}; do
             tag=${spec%%:*}; A=${spec#*:}; A=${A//,/ }
             timeout -k 10 500 python bench.py --topology mesh1m --steps ${M1M_STEPS:-3} --warmup 1 --cpu-sample 4 $A > "$OUT/m1m_$tag.json" 2> "$OUT/m1m_$tag.err"; rc=$?
             echo "m1m $tag rc=$rc $(python -c "import json; d=json.load(open('$OUT/m1m_$tag.json')); print(d['value'], d['ms_per_step'], d['parity_vs_cpu_sample'])" 2>/dev/null)"
             [ $rc -eq 0 ] || break
           done;;
    ksp2)  # KSP2 side bench: two PMC passes (3 KSP2 launches each), their sum, then the bench
           rc=0; i=0
           for P in FETCH_SIZE WRITE_SIZE; do
             i=$((i+1))
             timeout -s KILL 240 rocprofv3 --pmc $P -d "$OUT/kpmc$i" -o run --output-format csv -- \
               python scripts/bench_ksp2.py --steps 1 --warmup 0 --iso-reps 1 --no-cpu --no-lfa > "$OUT/kpmc$i.json" 2> "$OUT/kpmc$i.err"; rc=$?
             echo "ksp2 pmc $P rc=$rc"; [ $rc -eq 0 ] || break
           done
           if [ $rc -eq 0 ]; then
             ND=$(python -c "import json; print(json.load(open('$OUT/kpmc1.json'))['roofline']['destinations_per_launch'])")
             python scripts/pmc_sum.py "$OUT/kpmc1" "$OUT/kpmc2" --launches 3 --match "ospf::" --extra destinations_per_launch=$ND > "$OUT/ksp2_pmc.json" &&
             mkdir -p profiles/r06 && cp "$OUT/ksp2_pmc.json" profiles/r06/ksp2_pmc.json &&
             timeout -k 10 600 python scripts/bench_ksp2.py > "$OUT/ksp2.json" 2> "$OUT/ksp2.err"; rc=$?
             head -c 600 "$OUT/ksp2.json"; tail -3 "$OUT/ksp2.err"
           fi;;
    *) echo "unknown step $st"; rc=2;;
  esac
  echo "step $st rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
exit 0
