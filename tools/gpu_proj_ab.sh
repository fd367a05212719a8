#!/bin/bash
# Projection A/B (tools/proj_ab.py) on arxiv and Reddit, then the parity
# tests that run the Fin > 64 projection kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-p1}; VARS=${2:-"GAT_PROJ_X3=0;base"}
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/proj_ab.py --workload arxiv --variants "$VARS" > gpurun_out/proj_arxiv_${TAG}.json 2> gpurun_out/proj_arxiv_${TAG}.err &&
timeout -k 10 300 python3 tools/proj_ab.py --workload reddit --variants "$VARS" > gpurun_out/proj_reddit_${TAG}.json 2> gpurun_out/proj_reddit_${TAG}.err &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "proj_pipe or fullsize or arxiv or reddit or full" > gpurun_out/pytest_${TAG}.log 2>&1
echo "chain exit $?"
