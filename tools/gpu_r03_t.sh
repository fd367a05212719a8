#!/bin/bash
# arxiv / Reddit projection: store policy and residency A/B (is the loop-top
# vmcnt(0) on write-through stores what bounds k_project_wres / _x3?)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/proj_ab.py --workload arxiv --variants "base;GAT_STORE_WT=0;GAT_PROJ_WRES_WGS=2;GAT_PROJ_WRES_WGS=4;GAT_PROJ_WRES_WGS=1" > gpurun_out/proj_ab_arxiv_r03t.json 2>&1 &&
timeout -k 10 300 python3 tools/proj_ab.py --workload reddit --rounds 3 --variants "base;GAT_STORE_WT=0" > gpurun_out/proj_ab_reddit_r03t.json 2>&1
echo "chain exit $?"
