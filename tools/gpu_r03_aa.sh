#!/bin/bash
# default split rule: full GPU suite, smoke, emulated ranks, PPI bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r03aa}
mkdir -p gpurun_out
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $PYT -m gpu tests > gpurun_out/pytest_full_${TAG}.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 &&
timeout -k 10 300 python3 tools/emu_probe.py --workload ppi --ranks 2,4,8 --variants "base" > gpurun_out/emu_ppi_${TAG}.json 2>&1 &&
timeout -k 10 300 python3 bench.py --workloads arxiv,cifar,cifar_h8 --no-pmc --no-train --no-cpu-baseline > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err &&
timeout -k 10 200 tools/bwd_gather_probe > gpurun_out/bwd_gather_probe.json 2>&1
echo "chain exit $?"
