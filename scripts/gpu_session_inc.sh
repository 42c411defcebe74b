set -o pipefail
T=${TAG:-s33}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u scripts/bench_incremental.py > gpurun_out/$T/inc.jsonl 2> gpurun_out/$T/inc.err || { echo INC_FAIL; tail -20 gpurun_out/$T/inc.err; exit 1; }
cut -c1-420 gpurun_out/$T/inc.jsonl; tail -3 gpurun_out/$T/inc.err
