#!/bin/bash
# fused one-call forward: parity, host overhead, bench (PPI + small graphs), gap trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r03dd}
mkdir -p gpurun_out
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $PYT -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_gatnet.py > gpurun_out/pytest_${TAG}.log 2>&1 &&
timeout -k 10 120 python3 tools/host_overhead.py cifar > gpurun_out/host_${TAG}_cifar.txt 2>&1 &&
timeout -k 10 300 python3 bench.py --workloads arxiv,cifar,cifar_h8 --no-pmc --no-train --no-cpu-baseline --emulate-ranks '' > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err &&
bash tools/gpu_gap.sh ${TAG} ppi > gpurun_out/gap_${TAG}.log 2>&1
echo "chain exit $?"
