#!/bin/bash
# Bench evidence after the median-of-rounds kernel timings (the GPU suite of
# tools/gpu_r05y.sh ran at the same library): smoke, the default bench line,
# rocprofv3 kernel-trace stats of the bench and of the PPI-only bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=r05z
mkdir -p gpurun_out
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 &&
timeout -k 10 600 python3 bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- python3 bench.py --no-cpu-baseline --no-pmc > gpurun_out/prof_${TAG}.json 2> gpurun_out/prof_${TAG}.err &&
python3 tools/prof_summary.py gpurun_out/prof_${TAG}/run_kernel_stats.csv > gpurun_out/kernel_stats_bench_${TAG}.csv &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profppi_${TAG} -o run -- python3 bench.py --workloads '' --no-cpu-baseline --no-pmc --no-train --emulate-ranks '' > gpurun_out/profppi_${TAG}.json 2> gpurun_out/profppi_${TAG}.err &&
python3 tools/prof_summary.py gpurun_out/profppi_${TAG}/run_kernel_stats.csv > gpurun_out/kernel_stats_ppi_${TAG}.csv
echo "chain exit $?"
