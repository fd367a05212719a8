#!/bin/bash
# Edges per chunk for short rows: arxiv (7.9 per row) and CIFAR (9 per row)
# walk 2-3 chunks of U = 4; U = 8 covers a row in ~one chunk (one round of
# gathers in flight instead of two dependent ones).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05l
mkdir -p $O
for wl in arxiv cifar cifar_h8 ppi; do
  timeout -k 10 300 python3 tools/edge_ab.py --workload $wl --rounds 7 --iters 20 --layer \
    --variants "base;GAT_EDGE_U=8;GAT_EDGE_U=16" > $O/edge_ab_u_$wl.json 2> $O/edge_ab_u_$wl.err || exit 2
done
echo "chain exit 0"
