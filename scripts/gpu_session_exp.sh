set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/s26_exp.jsonl
: > $O
timeout -k 10 300 python -u scripts/exp_class.py --W 3 --n 2334 --order random >> $O 2> gpurun_out/s26_exp.err || { echo FAIL1; tail -20 gpurun_out/s26_exp.err; exit 1; }
timeout -k 10 300 python -u scripts/exp_class.py --W 3 --n 2334 --order locality >> $O 2>> gpurun_out/s26_exp.err || { echo FAIL2; tail -20 gpurun_out/s26_exp.err; exit 1; }
OSPF_MS_PACK=1 timeout -k 10 300 python -u scripts/exp_class.py --W 3 --n 2334 --order locality >> $O 2>> gpurun_out/s26_exp.err || { echo FAIL3; tail -20 gpurun_out/s26_exp.err; exit 1; }
timeout -k 10 300 python -u scripts/exp_class.py --W 56 --n 288 --order random >> $O 2>> gpurun_out/s26_exp.err || { echo FAIL4; exit 1; }
timeout -k 10 300 python -u scripts/exp_class.py --W 56 --n 288 --order locality >> $O 2>> gpurun_out/s26_exp.err || { echo FAIL5; exit 1; }
OSPF_MS_PACK=1 timeout -k 10 300 python -u scripts/exp_class.py --W 56 --n 288 --order locality >> $O 2>> gpurun_out/s26_exp.err || { echo FAIL6; exit 1; }
cat $O
