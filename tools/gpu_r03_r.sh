#!/bin/bash
# projection floors at arxiv and Reddit shapes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 120 tools/proj_floor 169343 128 > gpurun_out/proj_floor_arxiv.json 2>&1 &&
timeout -k 10 120 tools/proj_floor 232965 602 > gpurun_out/proj_floor_reddit.json 2>&1
echo "chain exit $?"
