#!/bin/bash
# Kernel-trace gap analysis of the eager layer step (tools/gap_probe.py) and the
# host enqueue cost, per workload.  usage: bash tools/gpu_gap.sh <tag> [workloads]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r03}
WLS=${2:-ppi}
mkdir -p gpurun_out
for W in $WLS; do
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gap_${TAG}_${W} -o run -- python3 tools/gap_probe.py run --workload $W --steps 200 > gpurun_out/gap_${TAG}_${W}.run.json 2> gpurun_out/gap_${TAG}_${W}.err &&
  python3 tools/gap_probe.py parse gpurun_out/gap_${TAG}_${W}/run_kernel_trace.csv > gpurun_out/gap_${TAG}_${W}.json || exit 1
  timeout -k 10 120 python3 tools/host_overhead.py $W > gpurun_out/host_${TAG}_${W}.txt 2>&1 || exit 1
done
echo "chain exit $?"
