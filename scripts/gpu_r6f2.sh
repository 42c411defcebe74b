#!/bin/bash
# round 6: the bench's first-run record with the unit-trace step's arguments
set -u
OUT=gpurun_out/r6_${1:-f2}; mkdir -p $OUT
for v in a fulldepth b; do
  case $v in
    fulldepth) E="OSPF_SWEEP_FULL_DEPTH=1";;
    *) E="";;
  esac
  timeout -k 10 300 env $E OSPF_SWEEP_TIMING=1 python bench.py --steps 5 --warmup 1 --no-cpu --iso-reps 3 > $OUT/b_$v.json 2> $OUT/b_$v.err || { tail -20 $OUT/b_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/b_$v.json')); print('$v', d['ms_per_step'], d['config']['root_classes']['first_sweep_after_graph_change'])"
done
