# Knob sweep of the multi-source BFS per width class (F100k, the bench's per-step counts).
set -o pipefail
T=${TAG:-s26}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/exp_class.py --W 3 --n 2334 --reps 3 --envs "" OSPF_MS_NB=112 OSPF_MS_NB=128 OSPF_MS_NB=160 OSPF_MS_PUSH_DIV=4 OSPF_MS_PUSH_DIV=16 OSPF_MS_PACK=1 > gpurun_out/$T/w3.jsonl 2> gpurun_out/$T/w3.err || { echo W3_FAIL; tail -20 gpurun_out/$T/w3.err; exit 1; }
cat gpurun_out/$T/w3.jsonl
timeout -k 10 400 python -u scripts/exp_class.py --W 1 --n 14003 --reps 3 --envs "" OSPF_MS_NB=110 OSPF_MS_NB=128 OSPF_MS_NB=224 OSPF_MS_PUSH_DIV=4 OSPF_MS_PUSH_DIV=16 > gpurun_out/$T/w1.jsonl 2> gpurun_out/$T/w1.err || { echo W1_FAIL; tail -20 gpurun_out/$T/w1.err; exit 1; }
cat gpurun_out/$T/w1.jsonl
timeout -k 10 400 python -u scripts/exp_class.py --W 56 --n 47 --reps 3 --envs "" OSPF_MS_PUSH_DIV=4 OSPF_MS_PUSH_DIV=16 OSPF_MS_PACK=1 OSPF_MS_R=32 > gpurun_out/$T/w56.jsonl 2> gpurun_out/$T/w56.err || { echo W56_FAIL; tail -20 gpurun_out/$T/w56.err; exit 1; }
cat gpurun_out/$T/w56.jsonl
