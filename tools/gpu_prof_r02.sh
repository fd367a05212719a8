#!/bin/bash
# Round-2 evidence: the bench command under rocprofv3 --kernel-trace --stats
# (PMC passes off: they run rocprofv3 themselves), condensed for profiles/.
# usage: bash tools/gpu_prof_r02.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r02}
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- python3 bench.py --no-pmc --no-cpu-baseline > gpurun_out/prof_${TAG}.json 2> gpurun_out/prof_${TAG}.err &&
python3 tools/prof_summary.py gpurun_out/prof_${TAG}/run_kernel_stats.csv > gpurun_out/kernel_stats_${TAG}.csv
echo "chain exit $?"
