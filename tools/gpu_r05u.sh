#!/bin/bash
# PPI edge kernel: output store policy (write-through / non-temporal) and its
# effect on the table's L2 hit rate; arxiv and CIFAR as controls.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05u
mkdir -p $O
for wl in ppi arxiv; do
  timeout -k 10 300 python3 tools/edge_ab.py --workload $wl --rounds 7 --iters 20 \
    --variants "base;GAT_STORE_WT=0;GAT_STORE_WT=2;GAT_STORE_WT=3" > $O/edge_ab_store_$wl.json 2> $O/edge_ab_store_$wl.err || exit 2
done
echo "chain exit 0"
