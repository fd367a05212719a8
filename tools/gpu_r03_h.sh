#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 120 tools/proj_floor > gpurun_out/proj_floor_ppi.json 2>&1
echo "chain exit $?"
