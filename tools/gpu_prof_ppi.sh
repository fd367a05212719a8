#!/bin/bash
# Headline-kernel evidence: the default PPI bench alone (no other workloads, no
# training object, no PMC, no CPU baseline) under rocprofv3 --kernel-trace
# --stats, so the edge kernel's average duration is PPI's only.
# usage: bash tools/gpu_prof_ppi.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r02}
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profppi_${TAG} -o run -- python3 bench.py --no-pmc --no-cpu-baseline --no-train --workloads ppi > gpurun_out/profppi_${TAG}.json 2> gpurun_out/profppi_${TAG}.err &&
python3 tools/prof_summary.py gpurun_out/profppi_${TAG}/run_kernel_stats.csv > gpurun_out/kernel_stats_ppi_${TAG}.csv
echo "chain exit $?"
