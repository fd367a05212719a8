#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r03d}
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/edge_ab.py --workload arxiv --variants "base;sched=1;GAT_WH_SLICES=2;GAT_WH_SLICES=4;GAT_WH_SLICES=8;GAT_WH_SLICES=8,GAT_EDGE_V=2;sched=1,GAT_WH_SLICES=8" > gpurun_out/ab_planes_${TAG}_arxiv.json 2>&1 &&
timeout -k 10 300 python3 tools/edge_ab.py --workload reddit_powerlaw --rounds 3 --variants "base;hubseg=4096;hubseg=8192" > gpurun_out/ab_hubseg_${TAG}.json 2>&1 &&
timeout -k 10 200 python3 tools/step_probe.py --workload ppi --variants "wk:;wres:GAT_PROJ_WRES=1" > gpurun_out/step_proj_${TAG}_ppi.json 2>&1
echo "chain exit $?"
