#!/bin/bash
# Training-step A/B (tools/train_ab.py) then the training GPU tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-t1}; W=${2:-reddit}; VARS=${3:-"base;GAT_WH_SLICES=1"}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_training.py tests/test_gpu_fullsize.py > gpurun_out/pytest_train_${TAG}.log 2>&1 &&
timeout -k 10 400 python3 tools/train_ab.py --workload $W --variants "$VARS" > gpurun_out/train_ab_${TAG}.json 2> gpurun_out/train_ab_${TAG}.err
echo "chain exit $?"
