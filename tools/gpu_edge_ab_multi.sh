#!/bin/bash
# Edge-kernel A/B on several workloads (tools/edge_ab.py, interleaved, graph-timed).
# usage: bash tools/gpu_edge_ab_multi.sh <tag> "<variants>" "<workloads>"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=$1; VARS=$2; WLS=${3:-"arxiv ppi cifar"}
mkdir -p gpurun_out
for W in $WLS; do
  timeout -k 10 300 python3 tools/edge_ab.py --workload $W --rounds 5 --iters 20 --variants "$VARS" > gpurun_out/ab_${W}_${TAG}.json 2> gpurun_out/ab_${W}_${TAG}.err || { echo "ab $W failed"; exit 1; }
done
echo "chain exit 0"
