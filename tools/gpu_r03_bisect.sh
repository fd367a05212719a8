#!/bin/bash
# source-pass bisection: the memory-only probe with the pass's pieces added
# one at a time, and the library's k_bwd_sources in a Reddit training step on
# the same box (rocprofv3 kernel stats)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r03bisect}
mkdir -p gpurun_out
timeout -k 10 300 ./tools/bwd_gather_probe > gpurun_out/bwd_bisect_${TAG}.json 2> gpurun_out/bwd_bisect_${TAG}.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/proftrain_${TAG} -o run -- python3 tools/train_ab.py --workload reddit --rounds 1 --steps 3 > gpurun_out/proftrain_${TAG}.json 2> gpurun_out/proftrain_${TAG}.err &&
python3 tools/prof_summary.py gpurun_out/proftrain_${TAG}/run_kernel_stats.csv > gpurun_out/kernel_stats_train_${TAG}.csv
echo "chain exit $?"
