#!/bin/bash
# Projection A/B (tools/proj_ab.py) on the listed workloads, then the parity
# tests that run the projection kernels.
# usage: bash tools/gpu_proj_ab.sh <tag> "<variants>" "<workloads, space separated>"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-p1}; VARS=${2:-"GAT_PROJ_X3=0;base"}; WLS=${3:-"arxiv reddit"}
mkdir -p gpurun_out
for W in $WLS; do
  timeout -k 10 300 python3 tools/proj_ab.py --workload $W --variants "$VARS" > gpurun_out/proj_${W}_${TAG}.json 2> gpurun_out/proj_${W}_${TAG}.err || { echo "proj_ab $W failed"; exit 1; }
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "proj or fast or full or arxiv or reddit" > gpurun_out/pytest_${TAG}.log 2>&1
echo "chain exit $?"
