#!/bin/bash
# Full GPU suite, smoke and the default bench line (no profilers).
# usage: bash tools/gpu_quick.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-quick}
mkdir -p gpurun_out
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $PYT -m gpu tests > gpurun_out/pytest_full_${TAG}.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 &&
timeout -k 10 600 python3 bench.py --detail-out gpurun_out/bench_detail_${TAG}.json > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err
echo "chain exit $?"
