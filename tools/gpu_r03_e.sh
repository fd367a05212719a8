#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r03e}
mkdir -p gpurun_out
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 1000 $PYT -m gpu tests > gpurun_out/pytest_full_${TAG}.log 2>&1 &&
timeout -k 10 400 python3 bench.py --no-pmc --no-train --no-cpu-baseline --emulate-ranks '' --workloads arxiv,cifar > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err &&
timeout -k 10 400 python3 tools/edge_ab.py --workload reddit_powerlaw --rounds 3 --variants "base;hublast=1" > gpurun_out/ab_hublast_${TAG}.json 2>&1
echo "chain exit $?"
