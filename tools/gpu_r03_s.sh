#!/bin/bash
# PPI: source-window passes (the plane's window fits an XCD's L2 at W >= 2)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/edge_ab.py --workload ppi --variants "base;passes=2;passes=3;passes=4" > gpurun_out/edge_ab_passes_ppi.json 2>&1
echo "chain exit $?"
