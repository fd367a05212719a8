#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/proj_ab.py --workload arxiv --variants "base;GAT_PROJ_WK_MAX=128,GAT_PROJ_WRES=0" > gpurun_out/proj_ab_arxiv_wk128.json 2>&1
echo "chain exit $?"
