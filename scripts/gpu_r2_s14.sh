set -o pipefail
T=${TAG:-r2s14}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u scripts/exp_msbfs.py --envs "" "OSPF_MS_NOMERGE=1" > $O/exp.jsonl 2> $O/exp.err || { echo EXP_FAIL; tail -20 $O/exp.err; exit 1; }
cat $O/exp.jsonl
