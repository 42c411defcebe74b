set -o pipefail
O=gpurun_out/r2s54
mkdir -p $O
export TMPDIR=/tmp
for env in "OSPF_X=0" "OSPF_DERIVE_CTILES=4" "OSPF_DERIVE_CTILES=16" "OSPF_DERIVE_CTILES=32" "OSPF_LV_NB=256"; do
  env $env timeout -k 10 300 python3 scripts/exp_derive.py --reps 2 --check 0 > $O/exp.json 2> $O/exp.err || { echo EXP_FAIL; tail -5 $O/exp.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/exp.json'));print('$env', [round(x,2) for x in d['phase1_ms']], {k:round(v,2) for k,v in d['median_phase2_ms'].items()})"
done
