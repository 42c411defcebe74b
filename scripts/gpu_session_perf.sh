# Rows-kernel block order experiment: per class, default vs batch-major.
set -o pipefail
T=${TAG:-s34}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
for c in 1:14003 3:2334 56:47; do
  timeout -k 10 300 python -u scripts/exp_class.py --W ${c%%:*} --n ${c##*:} --reps 3 --envs "" OSPF_ROWS_VMAJOR=1 >> gpurun_out/$T/cls.jsonl 2> gpurun_out/$T/cls.err || { echo CLS_FAIL; tail -20 gpurun_out/$T/cls.err; exit 1; }
done
cut -c1-200 gpurun_out/$T/cls.jsonl
