#!/bin/bash
# Where does the projection's in-step penalty come from?  step_probe with work
# inserted before each projection (PRED), and the projection run twice per step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r03g}
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/step_probe.py --workload ppi --double-proj --variants "base:;sleep:PRED=sleep;fill:PRED=fill;read:PRED=read;tinyproj:PRED=tinyproj" > gpurun_out/step_pred_${TAG}_ppi.json 2>&1 &&
timeout -k 10 200 python3 bench.py --workloads '' --no-pmc --no-train --no-cpu-baseline --emulate-ranks '' > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err
echo "chain exit $?"
