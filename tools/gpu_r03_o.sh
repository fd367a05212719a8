#!/bin/bash
# pipelined short-row edge kernels (U = 4/8, V = 1) A/B at PPI, arxiv, cifar_h8
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r03o}
mkdir -p gpurun_out
V="base;GAT_EDGE_PIPE=1;GAT_EDGE_PIPE=1,GAT_EDGE_U=8;GAT_EDGE_U=8"
for W in ppi arxiv cifar_h8; do
  timeout -k 10 200 python3 tools/edge_ab.py --workload $W --variants "$V" > gpurun_out/edge_ab_pipe_${W}_${TAG}.json 2>&1 || exit 1
done
echo "chain exit $?"
