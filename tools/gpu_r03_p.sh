#!/bin/bash
# dx kernel + distributed ping-pong: training and distributed GPU tests, smoke
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r03p}
mkdir -p gpurun_out
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $PYT -m gpu tests/test_gpu_training.py tests/test_gpu_distributed.py > gpurun_out/pytest_${TAG}.log 2>&1 &&
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 &&
timeout -k 10 300 python3 tools/train_ab.py --workload reddit --variants "base:" > gpurun_out/train_${TAG}_reddit.json 2>&1
echo "chain exit $?"
