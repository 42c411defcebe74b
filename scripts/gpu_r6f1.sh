#!/bin/bash
# round 6: the bench's first-sweep-after-change record in three settings
set -u
OUT=gpurun_out/r6_${1:-f1}; mkdir -p $OUT
for v in base noprobe fulldepth; do
  case $v in
    base) E=""; A="";;
    noprobe) E=""; A="--no-probe";;
    fulldepth) E="OSPF_SWEEP_FULL_DEPTH=1"; A="";;
  esac
  timeout -k 10 300 env $E python bench.py --cpu-sample 4 $A > $OUT/b_$v.json 2> $OUT/b_$v.err || { tail -20 $OUT/b_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/b_$v.json')); print('$v', d['ms_per_step'], d['config']['root_classes']['first_sweep_after_graph_change'])"
done
