#!/bin/bash
# two lane groups per row: parity, edge A/B at full size, per-rank shares
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r03z}
mkdir -p gpurun_out
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $PYT -m gpu tests/test_gpu_parity.py -k "split2 or pingpong" > gpurun_out/pytest_${TAG}.log 2>&1 &&
for W in ppi arxiv cifar_h8; do
  timeout -k 10 200 python3 tools/edge_ab.py --workload $W --variants "base;GAT_EDGE_SPLIT=2;GAT_EDGE_SPLIT=2,GAT_EDGE_U=8" > gpurun_out/edge_ab_split_${W}_${TAG}.json 2>&1 || exit 1
done &&
timeout -k 10 300 python3 tools/emu_probe.py --workload ppi --ranks 2,4,8 --variants "base;GAT_EDGE_SPLIT=2;GAT_EDGE_SPLIT=2,GAT_EDGE_U=8" > gpurun_out/emu_split_ppi_${TAG}.json 2>&1
echo "chain exit $?"
