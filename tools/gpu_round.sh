#!/bin/bash
# GPU tests + smoke, then the round's profiling evidence (gpu_profile_round.sh).
# usage: bash tools/gpu_round.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_${TAG}.log 2>&1 || { echo "pytest failed"; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 || { echo "smoke failed"; exit 1; }
bash tools/gpu_profile_round.sh ${TAG}
