# Multi-rank rehearsal of bench.py on ONE GPU (gloo collectives, every rank on
# device 0): checks the real partition / closure / gather code at N ranks on a
# full-size topology; timings are meaningless (ranks share the card).
# Usage: bash scripts/rehearse_ranks.sh <nranks> <topology> <outdir>
set -o pipefail
N=$1; TOPO=$2; O=$3
mkdir -p $O
PORT=$((20000 + RANDOM % 20000))
OPENR_BENCH_BACKEND=gloo OPENR_BENCH_SHARE_DEVICE=1 HSA_ENABLE_IPC_MODE_LEGACY=0 \
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
  --master-addr 127.0.0.1 --master-port $PORT bench.py --gpus $N --steps 1 --warmup 1 \
  --topology $TOPO --roots 0 --dist-parity 64 --iso-reps 1 > $O/rehearse_${N}_${TOPO}.json 2> $O/rehearse_${N}_${TOPO}.err
rc=$?
python3 -c "
import json,sys
d=json.loads([l for l in open('$O/rehearse_${N}_${TOPO}.json') if l.startswith('{')][0])
print('$TOPO', d['n_gpus'], d['config']['mode'], 'gathered', d['gathered_roots'], 'of', d['config']['n_nodes'], d['parity_vs_cpu_sample'])
" || { tail -20 $O/rehearse_${N}_${TOPO}.err; exit 1; }
exit $rc
