#!/bin/bash
# kernel stats of the Reddit training step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r03q}
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_train_${TAG} -o run -- python3 tools/train_ab.py --workload reddit --variants "base:" --rounds 1 > gpurun_out/kt_train_${TAG}.log 2>&1 &&
python3 tools/prof_summary.py gpurun_out/kt_train_${TAG}/run_kernel_stats.csv > gpurun_out/kt_train_${TAG}.csv
echo "chain exit $?"
