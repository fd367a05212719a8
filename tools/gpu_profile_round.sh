#!/bin/bash
# Round-end evidence on one GPU box: bench (default command), the same command
# under rocprofv3 --kernel-trace --stats, and PMC passes for the PPI and
# Reddit-scale edge kernels.  usage: bash tools/gpu_profile_round.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/prof_${TAG}.json 2> gpurun_out/prof_${TAG}.err || exit 1
python3 tools/prof_summary.py gpurun_out/prof_${TAG}/run_kernel_stats.csv > gpurun_out/kernel_stats_ppi_${TAG}.csv
bash tools/pmc_collect.sh ppi ${TAG} > gpurun_out/pmc_ppi_${TAG}.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --workload reddit --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_reddit_${TAG}.json 2> gpurun_out/bench_reddit_${TAG}.err || exit 1
bash tools/pmc_collect.sh reddit ${TAG} > gpurun_out/pmc_reddit_${TAG}.log 2>&1 || exit 1
echo done
