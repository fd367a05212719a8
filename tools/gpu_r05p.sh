#!/bin/bash
# Hub merge over a workgroup (k_edge_merge_wg) against the one-wave merge:
# hub parity tests, then the power-law Reddit layer A/B; and the PPI projection
# A/B of tools/gpu_r05o.sh.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05p
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -m gpu tests/test_gpu_hubs.py > $O/pytest_hubs.log 2>&1 || { tail -30 $O/pytest_hubs.log; exit 2; }
tail -1 $O/pytest_hubs.log
timeout -k 10 400 python3 tools/edge_ab.py --workload reddit_powerlaw --rounds 7 --iters 10 --layer \
  --variants "base;GAT_EDGE_MERGE=0" > $O/edge_ab_merge_powerlaw.json 2> $O/edge_ab_merge_powerlaw.err || exit 3
timeout -k 10 300 python3 tools/proj_bench.py --shapes "ppi,ppi@5632,arxiv" \
  --variants "base;GAT_PROJ_WRES=1;GAT_PROJ_WRES=1,GAT_PROJ_WRES_DIRECT=0" \
  --rounds 7 --out $O/proj_wres_ppi.json > $O/proj_wres_ppi.log 2>&1 || exit 4
echo "chain exit 0"
