#!/bin/bash
# ping-pong workspaces: parity + PPI bench; projection prototype floor probe
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r03i}
mkdir -p gpurun_out
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 120 tools/proj_floor > gpurun_out/proj_floor_${TAG}.json 2>&1


echo "chain exit $?"
