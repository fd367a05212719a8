#!/bin/bash
# Full GPU suite, smoke, then the default bench line.  Each step time-limited,
# chained with && (the first failure ends the call).
# usage: bash tools/gpu_full.sh <tag> [--no-bench]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r02}
mkdir -p gpurun_out
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $PYT -m gpu tests > gpurun_out/pytest_full_${TAG}.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 &&
if [ "$2" != "--no-bench" ]; then timeout -k 10 600 python bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err; fi
echo "chain exit $?"
