#!/bin/bash
# Power-law Reddit: where its extra time over uniform Reddit goes.  Edge-kernel
# knobs (pipelining, edges per chunk, hub split) on both graphs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05q
mkdir -p $O
for wl in reddit_powerlaw reddit; do
  timeout -k 10 500 python3 tools/edge_ab.py --workload $wl --rounds 5 --iters 10 \
    --variants "base;GAT_EDGE_PIPE=0;GAT_EDGE_U=8;GAT_HUB_SEG=1536" > $O/edge_ab_knobs_$wl.json 2> $O/edge_ab_knobs_$wl.err || exit 2
done
echo "chain exit 0"
