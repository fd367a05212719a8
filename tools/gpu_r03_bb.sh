#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 200 tools/bwd_gather_probe > gpurun_out/bwd_gather_probe.json 2>&1
echo "chain exit $?"
