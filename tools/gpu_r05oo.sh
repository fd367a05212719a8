#!/bin/bash
# Hub split shape A/B on power-law Reddit: equal-length segments per hub
# (GAT_HUB_BAL=1) and a lower split threshold (GAT_HUB_MIN), against the
# default (rows past 2 x 1024 edges cut into 1024-edge segments + a tail).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 500 python3 tools/edge_ab.py --workload reddit_powerlaw --rounds 5 --iters 5 \
  --variants "base;hubseg=1024;hubseg=1024,GAT_HUB_BAL=1;hubseg=1024,GAT_HUB_MIN=1024;hubseg=1024,GAT_HUB_MIN=1024,GAT_HUB_BAL=1;hubseg=1024,GAT_HUB_MIN=1536,GAT_HUB_BAL=1" \
  > $O/edge_ab_hubshape_powerlaw.json 2> $O/edge_ab_hubshape_powerlaw.err
echo "chain exit $?"
