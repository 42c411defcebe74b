set -o pipefail
O=gpurun_out/r2s43
mkdir -p $O
export TMPDIR=/tmp
bash scripts/rehearse_ranks.sh 4 fabric100k $O && bash scripts/rehearse_ranks.sh 4 fabric100k-w $O
