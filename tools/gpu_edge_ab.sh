#!/bin/bash
# Edge-kernel A/B on one workload (tools/edge_ab.py, interleaved, graph-timed),
# then one PMC pass (L2->fabric read requests, L2 hit/miss) per listed variant.
# usage: bash tools/gpu_edge_ab.sh <workload> <tag> "<variants; separated>"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
W=$1; TAG=$2; VARS=$3
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/edge_ab.py --workload $W --rounds 5 --variants "$VARS" > gpurun_out/ab_${TAG}.json 2> gpurun_out/ab_${TAG}.err || { echo "ab failed"; exit 1; }
IFS=';' read -ra VV <<< "$VARS"
for i in "${!VV[@]}"; do
  timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_128B_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmc_${TAG}_v$i -o run -- python3 tools/edge_ab.py --workload $W --variants "$VARS" --only $i --iters 3 > gpurun_out/pmc_${TAG}_v$i.log 2>&1 || { echo "pmc $i failed"; exit 1; }
done
echo "chain exit 0"
