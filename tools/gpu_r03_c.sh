#!/bin/bash
# r03 batch c: parity after the write-through projections, bench (no PMC), PPI trace gaps,
# power-law hub segment A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r03c}
mkdir -p gpurun_out
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $PYT tests/test_gpu_parity.py tests/test_gpu_fullsize.py > gpurun_out/pytest_parity_${TAG}.log 2>&1 &&
timeout -k 10 400 python3 bench.py --no-pmc --no-train --no-cpu-baseline --emulate-ranks '' --workloads reddit,arxiv,cifar > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err &&
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gap_${TAG}_ppi -o run -- python3 tools/gap_probe.py run --workload ppi --steps 200 > gpurun_out/gap_${TAG}_ppi.run.json 2> gpurun_out/gap_${TAG}_ppi.err &&
python3 tools/gap_probe.py parse gpurun_out/gap_${TAG}_ppi/run_kernel_trace.csv > gpurun_out/gap_${TAG}_ppi.json &&
timeout -k 10 400 python3 tools/edge_ab.py --workload reddit_powerlaw --rounds 3 --variants "base;hubseg=1024;hubseg=512;hubseg=256" > gpurun_out/ab_hubseg_${TAG}.json 2>&1
echo "chain exit $?"
