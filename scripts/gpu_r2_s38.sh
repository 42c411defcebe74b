set -o pipefail
T=${TAG:-r2s38}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for env in "OSPF_LV_MASKED=1" "OSPF_LV_MASKED=0" "OSPF_MS_PUSH_DIV=32" "OSPF_MS_PUSH_DIV=64" "OSPF_LV_NB=192" "OSPF_LV64=1"; do
  env $env timeout -k 10 300 python3 scripts/exp_derive.py --reps 3 --check 0 > $O/exp.json 2> $O/exp.err || { echo EXP_FAIL; tail -5 $O/exp.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/exp.json'));print('$env', [round(x,2) for x in d['phase1_ms']])"
done
