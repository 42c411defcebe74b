#!/bin/bash
# round 6: the first-run stall under rocprofv3's kernel trace, with and without the captured depth
set -u
OUT=gpurun_out/r6_${1:-f4}; mkdir -p $OUT; export TMPDIR=/tmp
for v in base fulldepth; do
  case $v in fulldepth) E="OSPF_SWEEP_FULL_DEPTH=1";; *) E="";; esac
  env $E timeout -k 10 420 rocprofv3 --kernel-trace --stats -d "$OUT/t_$v" -o run --output-format csv -- \
    python bench.py --steps 5 --warmup 1 --no-cpu --iso-reps 3 > $OUT/b_$v.json 2> $OUT/b_$v.err || { tail -20 $OUT/b_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/b_$v.json')); print('$v', d['ms_per_step'], d['config']['root_classes']['first_sweep_after_graph_change']['first_run_ms'])"
done
