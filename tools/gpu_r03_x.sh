#!/bin/bash
# per-rank edge passes at small shares: chunk length / rows per wave
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/emu_probe.py --workload ppi --ranks 2,4,8 --variants "base;GAT_EDGE_U=8;GAT_EDGE_U=16;GAT_EDGE_V=2" > gpurun_out/emu_ppi.json 2>&1
echo "chain exit $?"
