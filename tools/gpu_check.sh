#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprof kernel trace.
# Every GPU step has its own time limit; steps are chained with && so the
# first failure (or fault) ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r01}
timeout -k 10 480 python -m pytest tests -m gpu -q --maxfail=10 -p no:cacheprovider > gpurun_out/pytest_gpu_${TAG}.log 2>&1
echo "pytest exit $?" | tee -a gpurun_out/pytest_gpu_${TAG}.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/bench_${TAG}.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/prof_${TAG}.log 2>&1
echo "chain exit $?"
