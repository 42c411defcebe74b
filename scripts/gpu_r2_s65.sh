set -o pipefail
O=gpurun_out/r2s65
mkdir -p $O
export TMPDIR=/tmp
ALT=$PWD/openr_amd/lib/alt/libopenr_spf_hip.so
OPENR_SPF_ENGINE_SO=$ALT timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_derive.py tests/test_gpu_scale.py > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for env in "OPENR_SPF_ENGINE_SO=$ALT" "OSPF_X=0" "OPENR_SPF_ENGINE_SO=$ALT" "OSPF_X=0"; do
  env $env timeout -k 10 300 python3 scripts/exp_derive.py --reps 2 --check 16 > $O/exp.json 2> $O/exp.err || { echo EXP_FAIL; tail -5 $O/exp.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/exp.json'));print('${env##*/}', [round(x,2) for x in d['phase1_ms']], d['check_equal'])"
done
