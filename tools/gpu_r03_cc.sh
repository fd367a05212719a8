#!/bin/bash
# backward source pass with two float4s per lane: training tests, Reddit A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r03cc}
mkdir -p gpurun_out
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $PYT -m gpu tests/test_gpu_training.py > gpurun_out/pytest_train_${TAG}.log 2>&1 &&
timeout -k 10 600 python3 tools/train_ab.py --workload reddit --variants "v2u16:;v1u16:GAT_BWD_V=1;v2u8:GAT_BWD_U=8;v2u4:GAT_BWD_U=4;v1u8:GAT_BWD_V=1,GAT_BWD_U=8" > gpurun_out/train_ab_bwdv_${TAG}.json 2>&1
echo "chain exit $?"
