#!/bin/bash
# Hub segment length re-measured after the workgroup merge (k_edge_merge_wg):
# the merge's cost per segment fell, so shorter segments may now pay.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 500 python3 tools/edge_ab.py --workload reddit_powerlaw --rounds 5 --iters 5 --layer \
  --variants "base;hubseg=512;hubseg=768;hubseg=1536;hubseg=2048" \
  > $O/edge_ab_hubseg_wg_powerlaw.json 2> $O/edge_ab_hubseg_wg_powerlaw.err
echo "chain exit $?"
