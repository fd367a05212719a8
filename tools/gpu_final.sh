#!/bin/bash
# Round evidence: full GPU suite, smoke, the default bench line, the same
# command under rocprofv3 --kernel-trace --stats, the PPI-only bench under
# rocprofv3 (headline kernel stats), and the multi-GPU rehearsal at world 1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-final}
mkdir -p gpurun_out
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $PYT -m gpu tests > gpurun_out/pytest_full_${TAG}.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 &&
timeout -k 10 600 python3 bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- python3 bench.py --no-cpu-baseline --no-pmc > gpurun_out/prof_${TAG}.json 2> gpurun_out/prof_${TAG}.err &&
python3 tools/prof_summary.py gpurun_out/prof_${TAG}/run_kernel_stats.csv > gpurun_out/kernel_stats_bench_${TAG}.csv &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profppi_${TAG} -o run -- python3 bench.py --workloads '' --no-cpu-baseline --no-pmc --no-train --emulate-ranks '' > gpurun_out/profppi_${TAG}.json 2> gpurun_out/profppi_${TAG}.err &&
python3 tools/prof_summary.py gpurun_out/profppi_${TAG}/run_kernel_stats.csv > gpurun_out/kernel_stats_ppi_${TAG}.csv &&
timeout -k 10 400 python3 bench.py --dist --dist-workloads ppi,arxiv --steps 10 --warmup 3 > gpurun_out/bench_dist1_${TAG}.json 2> gpurun_out/bench_dist1_${TAG}.err
echo "chain exit $?"
