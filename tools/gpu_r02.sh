#!/bin/bash
# Round-2 GPU session: new-path tests first (hubs, sharded passes), then the
# full GPU suite, smoke, and the bench line.  Every GPU step has its own time
# limit; steps are chained with && so the first failure ends the call.
# usage: bash tools/gpu_r02.sh <tag> [pytest -k expr]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r02}
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $PYT -m gpu tests/test_gpu_hubs.py tests/test_gpu_distributed.py > gpurun_out/pytest_new_${TAG}.log 2>&1 &&
timeout -k 10 600 $PYT -m gpu tests --ignore=tests/test_gpu_hubs.py --ignore=tests/test_gpu_distributed.py -q > gpurun_out/pytest_rest_${TAG}.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 &&
timeout -k 10 600 python bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err
echo "chain exit $?"
