#!/bin/bash
# Selected GPU tests, then tools/emu_probe.py (per-rank compute of the
# partitioned step under knob / chunk variants).
# usage: bash tools/gpu_emu.sh <tag> "<pytest -k expr or empty>" <workload> <ranks> "<variants>"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-emu}; K=${2:-}; W=${3:-reddit}; R=${4:-8}; V=${5:-base}
mkdir -p gpurun_out
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests -k "$K" > gpurun_out/pytest_${TAG}.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_${TAG}.log; exit 1; }
  tail -2 gpurun_out/pytest_${TAG}.log
fi
timeout -k 10 600 python3 tools/emu_probe.py --workload $W --ranks $R --variants "$V" > gpurun_out/emu_${TAG}.json 2> gpurun_out/emu_${TAG}.err || { echo "emu failed"; tail -20 gpurun_out/emu_${TAG}.err; exit 1; }
cat gpurun_out/emu_${TAG}.json
