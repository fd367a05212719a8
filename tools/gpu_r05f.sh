#!/bin/bash
# PPI edge-kernel shape (U edges per chunk, V float4s per lane) re-checked at
# the round-5 kernel; hub order / segment length around the new default on
# power-law Reddit; kernel durations of the rank-share projections.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05f
mkdir -p $O
timeout -k 10 300 python3 tools/edge_ab.py --workload ppi --rounds 7 --iters 20 \
  --variants "base;GAT_EDGE_V=2;GAT_EDGE_U=8;GAT_EDGE_U=2;GAT_EDGE_V=2,GAT_EDGE_U=8" \
  > $O/edge_ab_uv_ppi.json 2> $O/edge_ab_uv_ppi.err || exit 2
timeout -k 10 400 python3 tools/edge_ab.py --workload reddit_powerlaw --rounds 5 --iters 5 \
  --variants "base;GAT_HUB_ORDER=hub;hubseg=768;hubseg=1536" \
  > $O/edge_ab_hub_powerlaw.json 2> $O/edge_ab_hub_powerlaw.err || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_share -o run -- \
  python3 tools/proj_bench.py --shapes "ppi@5632,arxiv@21184,ppi,arxiv" --rounds 2 \
  > $O/prof_share.txt 2>&1 || exit 2
python3 tools/prof_summary.py $O/prof_share/run_kernel_stats.csv > $O/kernel_stats_share.csv
echo "chain exit 0"
